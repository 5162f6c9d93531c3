"""PN frame-sync oracle (oracle/pn_oracle.c, restating rx_and_corr.cpp:332-392)
pinned on the CPU.  The reference correlator sits inside UHD_SAFE_MAIN next to
the radio calls (uhd, boost are absent) and has no tests or fixtures of its
own, so parity is pinned against an independent float64 numpy restatement of
the same loop: magnitudes within float32 rounding, identical decisions where
the threshold has margin, the reference's early-exit order (first channel,
then first lag), and the copy_buff / copy_to_shared_mem frame layout."""
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
