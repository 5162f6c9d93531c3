"""PN frame-sync oracle (oracle/pn_oracle.c, restating rx_and_corr.cpp:332-392)
pinned on the CPU.  The reference correlator sits inside UHD_SAFE_MAIN next to
the radio calls (uhd, boost are absent) and has no tests or fixtures of its
own, so parity is pinned against an independent float64 numpy restatement of
the same loop: magnitudes within float32 rounding, identical decisions where
the threshold has margin, the reference's early-exit order (first channel,
then first lag), and the copy_buff / copy_to_shared_mem frame layout."""
import os

import numpy as np
import pytest

from pn_cases import rx_buffer


def np_mags(buf, pn):
    R, N = buf.shape
    L = pn.size
    nl = N - L + 1
    out = np.zeros((R, max(nl, 0)))
    for ch in range(R):
        x = buf[ch].astype(np.complex128)
        # temp[i] = sum_j pn[j] * x[i+j]  (no conjugate)
        out[ch] = np.abs(np.correlate(x, np.conj(pn.astype(np.complex128)), "valid")) / L
    return out


@pytest.mark.parametrize("R,N,L", [(1, 600, 63), (3, 2000, 255), (2, 1500, 1023)])
def test_oracle_mags_match_float64(oracle, R, N, L):
    buf, pn = rx_buffer(R, N, L, {R - 1: ((N - L) // 2, 0.8 - 0.3j)})
    pos, mag = oracle.pn_correlate(buf, pn, 0.5, mag=True)
    ref = np_mags(buf, pn)
    assert mag.shape == ref.shape
    assert np.abs(mag - ref).max() <= 1e-5 * max(1.0, ref.max())
    nl = N - L + 1
    first = np.flatnonzero(ref.ravel() >= 0.5)
    assert pos == first[0] and pos == (R - 1) * nl + (N - L) // 2


def test_oracle_early_exit_order(oracle):
    R, N, L = 4, 3000, 127
    # hits in channels 1 and 3; channel 1's is later in time but earlier in the search order
    buf, pn = rx_buffer(R, N, L, {1: (2500, 1.0), 3: (100, 1.2)})
    nl = N - L + 1
    pos, _ = oracle.pn_correlate(buf, pn, 0.5)
    assert pos == 1 * nl + 2500
    pos_full, mag = oracle.pn_correlate(buf, pn, 0.5, mag=True)
    assert pos_full == pos
    # threshold above every lag: no hit, like the reference's `continue`
    pos, _ = oracle.pn_correlate(buf, pn, float(mag.max()) * 1.01)
    assert pos == -1
    # threshold exactly equal to a lag's value: that lag (>=) is the hit
    t3 = float(mag[3].max())  # only channel 3 reaches it, at its peak
    pos, _ = oracle.pn_correlate(buf, pn, t3)
    assert pos == 3 * nl + int(np.argmax(mag[3]))
    t = float(mag[1].max())
    pos, _ = oracle.pn_correlate(buf, pn, t)
    assert pos == 1 * nl + int(np.flatnonzero(mag[1] >= t)[0])
    t_up = float(np.nextafter(np.float32(t), np.float32(np.inf)))
    pos, _ = oracle.pn_correlate(buf, pn, t_up)
    assert pos == 3 * nl + int(np.flatnonzero(mag[3] >= t_up)[0])


def test_oracle_short_buffer(oracle):
    buf, pn = rx_buffer(2, 50, 63, {})
    assert oracle.pn_correlate(buf, pn, 0.0)[0] == -1


@pytest.mark.parametrize("lag", [0, 1, 777])
def test_oracle_extract_layout(oracle, lag):
    """copy_buff[ch] = buff1[ch][lag+L:] ++ buff2[ch][:lag] (rx_and_corr.cpp:370-392);
    symbol s of channel ch = copy_buff[ch][s*(C+cp)+cp : s*(C+cp)+cp+C] (64-87)."""
    R, N, L, C, cp = 3, 5000, 127, 256, 32
    rng = np.random.default_rng(lag)
    b1 = (rng.standard_normal((R, N)) + 1j * rng.standard_normal((R, N))).astype(np.complex64)
    b2 = (rng.standard_normal((R, N)) + 1j * rng.standard_normal((R, N))).astype(np.complex64)
    nsym = (N - L) // (C + cp)
    got = oracle.pn_extract(b1, b2, L, lag, C, cp, nsym)
    for ch in range(R):
        seq = np.concatenate([b1[ch, lag + L:], b2[ch, :lag]])
        assert seq.size == N - L
        for s in range(nsym):
            assert np.array_equal(got[s, ch], seq[s * (C + cp) + cp: s * (C + cp) + cp + C])


# ----------------------------------------------- pinned to the reference loop

REF_PN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                      "libref_pn.so")


def _ref_pn():
    import ctypes
    L = ctypes.CDLL(REF_PN)
    L.ref_pn_correlate.restype = ctypes.c_longlong
    L.ref_pn_correlate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
    return L


def ref_search(lib, buf, pn, thres):
    """The reference's own correlator block (rx_and_corr.cpp:329-360, built by
    oracle/build_ref.sh), one channel at a time in the reference's channel
    order -> (ch * (N-L+1) + lag, |corr|/L at the hit) or (-1, None)."""
    import ctypes
    R, N = buf.shape
    nl = N - pn.size + 1
    for ch in range(R):
        row = np.ascontiguousarray(buf[ch:ch + 1])
        m = ctypes.c_float(0.0)
        lag = lib.ref_pn_correlate(row.ctypes.data, 1, N, pn.ctypes.data, pn.size, thres, ctypes.byref(m))
        if lag >= 0:
            return ch * nl + lag, m.value
    return -1, None


@pytest.mark.skipif(not os.path.exists(REF_PN), reason="oracle/_ref/libref_pn.so not built (needs /root/reference)")
@pytest.mark.parametrize("R,N,L,hits,seed", [(1, 600, 63, {0: (200, 0.9)}, 1),
                                             (3, 2000, 255, {2: (1000, 0.8 - 0.3j)}, 2),
                                             (4, 3000, 127, {1: (2500, 1.0), 3: (100, 1.2)}, 3),
                                             (2, 1500, 1023, {0: (0, 0.7j), 1: (477, 1.1)}, 4),
                                             (2, 900, 1, {}, 5)])
def test_oracle_bitexact_vs_reference_loop(oracle, R, N, L, hits, seed):
    """The oracle's hit index and magnitude equal the reference block's own, bit
    for bit, at thresholds taken from the lags' own values (ties decide with
    >=), one ulp above and below, and above every lag (no hit)."""
    lib = _ref_pn()
    buf, pn = rx_buffer(R, N, L, hits, seed=seed)
    pn = np.ascontiguousarray(pn, np.complex64)
    _, mag = oracle.pn_correlate(buf, pn, 0.0, mag=True)
    flat = np.sort(mag.ravel())
    picks = [flat[-1], flat[-2], flat[len(flat) // 2], flat[len(flat) // 7]]
    thresholds = []
    for t in picks:
        t = np.float32(t)
        thresholds += [t, np.nextafter(t, np.float32(np.inf)), np.nextafter(t, np.float32(-np.inf))]
    thresholds.append(np.nextafter(np.float32(flat[-1]), np.float32(np.inf)))
    for t in thresholds:
        pos, m = oracle.pn_correlate(buf, pn, float(t), mag=True)
        rpos, rmag = ref_search(lib, buf, pn, float(t))
        assert pos == rpos, (t, pos, rpos)
        if rpos >= 0:
            nl = N - L + 1
            assert np.float32(m[rpos // nl, rpos % nl]) == np.float32(rmag)
