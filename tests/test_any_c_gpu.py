"""FFT lengths beyond the powers of two (fft_any.hip): the reference transforms
whatever `dimension` it is built with (ShMemSymBuff.hpp:47) through FFTW /
cuFFT, so the library takes any C in [2, 8192] -- LTE's 1536, 600 and 1200,
odd and prime lengths, 8192.  Checked through the C ABI against numpy
(float64 FFT) and the oracle (its mixed-radix float64 DFT + the cpuLS.hpp
LS / MRC restatement); tolerance helpers.RTOL = 1e-5 norm- and element-wise."""
import numpy as np
import pytest

from helpers import parity

pytestmark = pytest.mark.gpu

SIZES = [2, 3, 5, 6, 12, 15, 100, 243, 600, 1021, 1200, 1536, 2047, 3000, 4095, 6144, 8192]


def to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def qpsk(K, seed=7):
    rng = np.random.default_rng(seed)
    a = np.float32(0.70710678)
    return (rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)


@pytest.mark.parametrize("C", SIZES)
def test_fft_rows_any_c_vs_numpy(ofdm, dev, C):
    rng = np.random.default_rng(C)
    n = 37
    x = (rng.standard_normal((n, C)) + 1j * rng.standard_normal((n, C))).astype(np.complex64)
    d = to_dev(x, dev)
    out = ofdm.c64(x.shape, dev)
    tol = 2e-6 * max(np.log2(C), 1.0)
    got = host(ofdm.fft_rows(d, out))
    ref = np.fft.fft(x.astype(np.complex128), axis=-1)
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max()
    inv = host(ofdm.fft_rows(d, out, inverse=True))
    refi = np.fft.ifft(x.astype(np.complex128), axis=-1) * C
    assert np.abs(inv - refi).max() <= tol * np.abs(refi).max()
    assert np.array_equal(host(ofdm.fft_rows(d)), got)  # in place


def test_fft_rows_any_c_many_rows(ofdm, dev):
    """More row groups than the persistent grid (2048 workgroups x G rows)."""
    C = 12  # G = 341 rows per workgroup
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((2048 * 341 + 77, C)) + 1j * rng.standard_normal((2048 * 341 + 77, C))).astype(
        np.complex64)
    got = host(ofdm.fft_rows(to_dev(x, dev)))
    ref = np.fft.fft(x.astype(np.complex128), axis=-1)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("C,R,prefix", [(6, 3, 0), (12, 1, 3), (128, 5, 9), (128, 64, 32), (256, 7, 18), (256, 64, 0),
                                        (512, 1, 0), (512, 32, 36), (600, 4, 44), (1021, 3, 0), (1200, 8, 84),
                                        (1536, 8, 108), (1536, 64, 0), (3000, 2, 0), (3072, 3, 0), (3072, 16, 216),
                                        (6144, 4, 432), (6144, 12, 0),
                                        (8192, 2, 512)])
def test_frame_demod_any_c_vs_oracle(ofdm, oracle, dev, C, R, prefix):
    F, S = 2, 4
    X = to_dev(qpsk(C - 1), dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=C + R)
    out = host(ofdm.frame_demod(iq, X, prefix))
    ref = oracle.frames_demod(host(iq), host(X), prefix)
    parity(out, ref)
    # the synthetic frames decode to their own QPSK symbols
    assert int(ofdm.count_symbol_errors(to_dev(out, dev), S, seed=C + R).item()) == 0
    # estimate + combine (the staged two-call flow) gives the same bytes
    ws = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_estimate(iq, X, prefix, ws)
    out2 = ofdm.c64(out.shape, dev)
    ofdm.frame_combine(iq, prefix, ws, out2)
    assert np.array_equal(host(out2), out)


@pytest.mark.parametrize("C,R", [(7, 2), (601, 5), (1023, 8), (1535, 3)])
def test_odd_c_freq_demod_vs_oracle(ofdm, oracle, dev, C, R):
    """Odd C = even K: shiftOneRow's memmoves leave the last output in place
    (cpuLS.hpp:135-149) -- the one-bin-per-lane combine and out_pos_any."""
    F, S = 3, 5
    X = to_dev(qpsk(C - 1), dev)
    Y = ofdm.synth_frames(F, S, R, C, X, seed=C, freq_domain=True)
    out = host(ofdm.frame_demod_freq(Y, X))
    parity(out, oracle.frames_demod_freq(host(Y), host(X)))
    assert int(ofdm.count_symbol_errors(to_dev(out, dev), S, seed=C).item()) == 0


@pytest.mark.parametrize("C,R", [(7, 1), (12, 3), (1536, 16), (1023, 4)])
def test_stages_any_c_vs_oracle(ofdm, oracle, dev, C, R):
    rng = np.random.default_rng(C * R)
    K = C - 1
    X = qpsk(K)
    Yp = (rng.standard_normal((R, C)) + 1j * rng.standard_normal((R, C))).astype(np.complex64)
    Hc_ref, P_ref = oracle.ls(Yp, X)
    Hc, P = ofdm.ls_estimate(to_dev(Yp, dev), to_dev(X, dev))
    parity(host(Hc), Hc_ref)
    parity(host(P), P_ref)
    Yd = (rng.standard_normal((4, R, C)) + 1j * rng.standard_normal((4, R, C))).astype(np.complex64)
    out = host(ofdm.mrc_demod(to_dev(Yd, dev), Hc, P))
    parity(out, np.stack([oracle.mrc(Yd[s], Hc_ref, P_ref) for s in range(4)]))
    # the per-stage gpuLS kernels: product, combine + rotate, shift
    prod = ofdm.channel_conj_product(to_dev(Yd, dev), Hc)
    comb = host(ofdm.combine_products(prod, P))
    parity(comb, np.stack([oracle.mrc(Yd[s], Hc_ref, P_ref) for s in range(4)]))
    rows = (rng.standard_normal((3, K)) + 1j * rng.standard_normal((3, K))).astype(np.complex64)
    assert np.array_equal(host(ofdm.shift_rows(to_dev(rows, dev))),
                          np.stack([oracle.shift_one_row(r) for r in rows]))


@pytest.mark.parametrize("C,R,prefix", [(128, 7, 9), (256, 10, 18), (512, 7, 36), (1536, 6, 16), (3072, 5, 24), (6144, 4, 40), (1200, 3, 0)])
def test_estimate_export_and_antenna_partials_any_c(ofdm, oracle, dev, C, R, prefix):
    """The estimate of a non-fused size (C = 128 ... 6144: the lane orders of
    frame_td_fft512.hip; 1200: the bin layout) exported to the reference layout
    matches the oracle's LS; the antenna-split partials (numerators + |H|^2)
    summed over two shards and finalised give the full receiver's output."""
    F, S = 2, 4
    X = to_dev(qpsk(C - 1), dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=C + 3)
    ws = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_estimate(iq, X, prefix, ws)
    H, P = ofdm.frame_export_estimate(ws, F, S, R, C, frame=1)
    Y0 = oracle.fft_rows(host(iq)[1, 0, :, prefix:])
    H_ref, P_ref = oracle.ls(Y0, host(X))
    parity(host(H), H_ref)
    parity(host(P), P_ref)
    full = host(ofdm.frame_demod(iq, X, prefix))
    import torch
    num, psum = None, None
    for r0, r1 in ((0, R // 2), (R // 2, R)):
        part = iq[:, :, r0:r1].contiguous()
        Pp, wsp = ofdm.frame_ls_partial(part, X, prefix)
        n = ofdm.frame_mrc_partial(part, wsp, prefix)
        num = n if num is None else num + n
        psum = Pp if psum is None else psum + Pp
    K = C - 1
    out = ofdm.c64((F, S - 1, K), dev)
    ofdm.mrc_finalize(num.reshape(-1), 0, S - 1, K, psum.reshape(-1).contiguous(), out)
    torch.cuda.synchronize()
    parity(host(out), full)


@pytest.mark.parametrize("C", [128, 256, 512, 1536, 3072, 6144, 600])
@pytest.mark.parametrize("F,S,R,prefix", [(1, 2, 1, 0), (3, 2, 2, -1), (2, 9, 1, 7)])
def test_small_batches_any_c_vs_oracle(ofdm, oracle, dev, C, F, S, R, prefix):
    """Edge shapes of the fused non-power-of-two receivers: one data symbol per
    frame, a single antenna, fewer symbols than waves, a cyclic prefix as long
    as the symbol (prefix = -1 -> C) and an odd one.  With R = 1 nothing is
    combined: a Rayleigh deep-fade bin divides by |H|^2 ~ 1e-4, which turns the
    f32 FFT's ~1e-7 absolute error into ~1e-5 of that output, so the
    element-wise bound is 1e-4 there (norm-relative stays 1e-5)."""
    prefix = C if prefix < 0 else prefix
    X = to_dev(qpsk(C - 1), dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=C + F + R)
    out = host(ofdm.frame_demod(iq, X, prefix))
    parity(out, oracle.frames_demod(host(iq), host(X), prefix), erel_tol=1e-4 if R == 1 else None)
    if R > 1:  # one antenna has no diversity: a deep fade under the noise flips a decision (so does the oracle)
        assert int(ofdm.count_symbol_errors(to_dev(out, dev), S, seed=C + F + R).item()) == 0


@pytest.mark.parametrize("C,lane", [(512, True), (600, False), (1024, True)])
def test_combine_freq_and_estimate_layouts(ofdm, dev, C, lane):
    """at the sizes with a fused receiver (lane-order estimates)
    the time- and frequency-domain stage pairs refuse each other's
    workspaces; at other sizes (600) both estimates are in the bin layout
    and each combine accepts the other's estimate with the same result."""
    F, S, R = 2, 3, 4
    X = to_dev(qpsk(C - 1), dev)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=3, noise_std=0.02)
    Y = ofdm.fft_rows(iq.clone())
    ref = host(ofdm.frame_demod(iq, X, 0))
    ws = ofdm.workspace(F, S, R, C, dev)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    ofdm.frame_estimate(iq, X, 0, ws)
    if lane:
        with pytest.raises(ofdm.OfdmError, match="lane order"):
            ofdm.frame_combine_freq(Y, ws, out)
    else:
        ofdm.frame_combine_freq(Y, ws, out)
        parity(host(out), ref)
    ofdm.frame_estimate_freq(Y, X, ws)
    if lane:
        with pytest.raises(ofdm.OfdmError, match="frequency-domain estimate"):
            ofdm.frame_combine(iq, 0, ws, out)
    else:
        ofdm.frame_combine(iq, 0, ws, out)
        parity(host(out), ref)
