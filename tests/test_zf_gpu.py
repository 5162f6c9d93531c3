"""Zero forcing on the GPU (ofdm_zf_precoder / _transpose / _apply / _detect,
SURVEY.md 8(f) rank 4) against the oracle restatement of
createZeroForcingMatrix / multiplyWithChannelInv (cpuLS.hpp:400-463).

Tolerances (floating point, written here as the north_star asks):
  * precoder: the reference inverts G = A A^H with LAPACK cgetrf + cgetri;
    the oracle restates that LU algorithm and the GPU computes it in the same
    order (every element accumulated in the oracle's order, no fused
    multiply-adds, Smith's reciprocal on both sides): bit-identical;
  * apply / detect: the same sums in a different association (FMA
    contraction): norm-relative <= 1e-5 AND element-wise <= 1e-5 relative
    with the output RMS as floor (helpers.parity, the receiver's bound);
  * transpose and the two output layouts of the precoder: bit-equal.
At full size (20k symbols x 1023 subcarriers) the size-independent
properties: uplink ZF detection and precoded downlink both return the QPSK
symbols (norm-relative <= 1e-4, zero hard-decision errors)."""
import numpy as np
import pytest

from helpers import parity
from zf_cases import channel, qpsk, rel_err, rel_err_per_subcarrier

pytestmark = pytest.mark.gpu


def dev_t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("U,R,K", [(1, 1, 5), (4, 16, 1023), (16, 64, 1023), (32, 64, 255),
                                   (32, 256, 64), (8, 1024, 16), (3, 7, 100), (2, 2, 1)])
def test_zf_precoder_parity(ofdm, oracle, dev, U, R, K):
    H = channel(U, R, K, seed=U * 7 + R + K)
    ref = oracle.zf_precoder(H)
    W, Wt = ofdm.zf_precoder(dev_t(H, dev))
    W, Wt = W.cpu().numpy(), Wt.cpu().numpy()
    assert np.array_equal(W, ref), f"max per-subcarrier rel. err {rel_err_per_subcarrier(W, ref):.2e}"
    assert np.array_equal(Wt, W.transpose(1, 2, 0))
    Wt2 = ofdm.zf_transpose(dev_t(W, dev)).cpu().numpy()
    assert np.array_equal(Wt2, Wt)


def test_zf_precoder_single_output(ofdm, dev):
    H = dev_t(channel(4, 8, 33, seed=3), dev)
    W_only, none = ofdm.zf_precoder(H, Wt=False)
    assert none is None
    none, Wt_only = ofdm.zf_precoder(H, W=False)
    assert none is None
    assert np.array_equal(Wt_only.cpu().numpy(), W_only.cpu().numpy().transpose(1, 2, 0))


# The shapes select every kernel of the shape-based dispatch (zf.hip
# gemm_dispatch): detect -- register tiles (U <= 8 or R < 8), W-stationary
# MFMA (U > 8, R <= 72), 8-wave MFMA (U > 16, R > 72), 128-subcarrier MFMA
# (8 < U <= 16, R > 72); apply -- 16-B-lane W-stationary tiles (R >= 8 and
# K >= 2: 8-row tiles for U <= 20, 4-row tiles for U <= 40; K odd exercises the
# lane that stores subcarrier K-1 alone), register tiles (R < 8 or K < 2).
@pytest.mark.parametrize("U,R,K,n", [(1, 1, 5, 1), (2, 4, 1023, 7), (3, 5, 64, 9), (4, 16, 1023, 33),
                                     (5, 12, 130, 17), (8, 64, 1023, 40), (12, 40, 200, 16),
                                     (16, 64, 1023, 100), (17, 64, 65, 3), (32, 64, 255, 25),
                                     (16, 100, 1023, 8), (24, 100, 130, 20)])
def test_zf_apply_detect_parity(ofdm, oracle, dev, U, R, K, n):
    H = channel(U, R, K, seed=n)
    W = oracle.zf_precoder(H)
    X = qpsk(n, U, K, seed=n + 1)
    Y = oracle.zf_apply(W, X)
    Wt = ofdm.zf_transpose(dev_t(W, dev))
    got_Y = ofdm.zf_apply(Wt, dev_t(X, dev)).cpu().numpy()
    assert rel_err(got_Y, Y) < 1e-5
    parity(got_Y, Y)  # norm-wise and element-wise, 1e-5
    Yn = (Y + 0.05 * qpsk(n, R, K, seed=n + 2)).astype(np.complex64)  # not just W X
    got_X = ofdm.zf_detect(Wt, dev_t(Yn, dev)).cpu().numpy()
    ref_X = oracle.zf_detect(W, Yn)
    assert rel_err(got_X, ref_X) < 1e-5
    parity(got_X, ref_X)


def test_cpuls_zf_call_sequence(oracle, dev, tmp_path):
    """createZeroForcingMatrix + multiplyWithChannelInv through the drop-in
    cpuLS.hpp (a C++ driver, tests/cpp/zf_driver.cpp): W in the reference's
    H layout, X left rotCube'd in place, HX = W x for one symbol."""
    from test_zf_cpu import build_zf_driver
    import subprocess
    R, cols, U = 16, 257, 4
    K = cols - 1
    H = channel(U, R, K, seed=31)
    x = qpsk(1, U, K, seed=32)[0]
    H.tofile(tmp_path / "H.bin")
    x.tofile(tmp_path / "X.bin")
    exe = build_zf_driver(str(tmp_path))
    subprocess.run([exe, str(R), str(cols), str(U)], cwd=tmp_path, check=True, timeout=120)
    W = np.fromfile(tmp_path / "W.bin", np.complex64).reshape(K, U, R)
    ref = oracle.zf_precoder(H)
    assert np.array_equal(W, ref)
    Xrot = np.fromfile(tmp_path / "Xrot.bin", np.complex64)
    assert np.array_equal(Xrot, H.transpose(2, 1, 0).ravel())  # [col][row][user]
    HX = np.fromfile(tmp_path / "HX.bin", np.complex64).reshape(R, K)
    assert rel_err(HX, oracle.zf_apply(W, x[None])[0]) < 1e-5


def test_zf_empty_and_limits(ofdm, dev):
    import torch
    Wt = torch.zeros((4, 8, 16), dtype=torch.complex64, device=dev)
    X = torch.zeros((0, 4, 16), dtype=torch.complex64, device=dev)
    assert ofdm.zf_apply(Wt, X).shape == (0, 8, 16)
    Y = torch.zeros((0, 8, 16), dtype=torch.complex64, device=dev)
    assert ofdm.zf_detect(Wt, Y).shape == (0, 4, 16)
    H0 = torch.zeros((4, 8, 0), dtype=torch.complex64, device=dev)
    ofdm.zf_precoder(H0)
    with pytest.raises(ofdm.OfdmError, match="users"):
        ofdm.zf_precoder(torch.zeros((33, 64, 4), dtype=torch.complex64, device=dev))
    with pytest.raises(ofdm.OfdmError, match="users\\*rows"):
        ofdm.zf_precoder(torch.zeros((16, 513, 4), dtype=torch.complex64, device=dev))


def test_zf_full_size_round_trips(ofdm, dev):
    """U = 16 users, R = 64 antennas, 1023 subcarriers, 20 000 symbols."""
    import torch
    U, R, K, n = 16, 64, 1023, 20000
    H = dev_t(channel(U, R, K, seed=21), dev)
    _, Wt = ofdm.zf_precoder(H, W=False)
    g = torch.Generator(device=dev)
    g.manual_seed(22)
    b = torch.randint(0, 2, (2, n, U, K), device=dev, generator=g).to(torch.float32) * 2 - 1
    X = torch.complex(b[0], b[1]) * np.sqrt(0.5)
    del b
    Hc = torch.conj(H).resolve_conj().contiguous()  # Wt-layout of the uplink channel A^H
    up = ofdm.zf_apply(Hc, X)  # y = A^H x
    Xh = ofdm.zf_detect(Wt, up)
    err = (torch.linalg.vector_norm(Xh - X) / torch.linalg.vector_norm(X)).item()
    assert err < 1e-4
    dec = lambda z: (torch.sign(z.real) != torch.sign(X.real)) | (torch.sign(z.imag) != torch.sign(X.imag))
    assert int(dec(Xh).sum().item()) == 0
    down = ofdm.zf_detect(Hc, ofdm.zf_apply(Wt, X))  # sum_r A(u, r) (W x)_r
    err = (torch.linalg.vector_norm(down - X) / torch.linalg.vector_norm(X)).item()
    assert err < 1e-4
    assert int(dec(down).sum().item()) == 0


@pytest.mark.parametrize("U,R,K,n,ldy,ldx", [(16, 64, 1023, 40, 1024, 1024), (16, 64, 1023, 33, 1023, 1024),
                                             (16, 64, 1023, 20, 1030, 1023), (4, 16, 1023, 9, 1024, 1040),
                                             (24, 40, 200, 16, 208, 201), (9, 72, 65, 70, 80, 72)])
def test_zf_detect_pitched(ofdm, oracle, dev, U, R, K, n, ldy, ldx):
    """ofdm_zf_detect_ex on row-padded layouts: the first K columns of every
    row read and written, the pad untouched (NaN-filled input pad, NaN
    sentinels in the output pad), the result against the oracle at the
    detect's 1e-5 bound -- and bit-identical to the unpadded detect where
    both run the W-stationary kernel (U > 8, R <= 72)."""
    import torch
    H = channel(U, R, K, seed=n + 5)
    W = oracle.zf_precoder(H)
    Yn = (oracle.zf_apply(W, qpsk(n, U, K, seed=n + 6)) + 0.05 * qpsk(n, R, K, seed=n + 7)).astype(np.complex64)
    ref = oracle.zf_detect(W, Yn)
    Wt = ofdm.zf_transpose(dev_t(W, dev))
    Yp = torch.full((n, R, ldy), float("nan"), dtype=torch.complex64, device=dev)
    Yp[:, :, :K] = dev_t(Yn, dev)
    out = torch.full((n, U, ldx), float("nan"), dtype=torch.complex64, device=dev)
    ofdm.zf_detect_pitched(Wt, Yp, out=out)
    got = out.cpu().numpy()
    assert np.isnan(got[:, :, K:]).all()
    parity(got[:, :, :K], ref)
    if U > 8:
        assert np.array_equal(got[:, :, :K], ofdm.zf_detect(Wt, dev_t(Yn, dev)).cpu().numpy())


def test_zf_detect_pitched_limits(ofdm, dev):
    import torch
    Wt = torch.zeros((4, 100, 16), dtype=torch.complex64, device=dev)
    Y = torch.zeros((2, 100, 32), dtype=torch.complex64, device=dev)
    with pytest.raises(ofdm.OfdmError, match="rows <= 72"):
        ofdm.zf_detect_pitched(Wt, Y)
    Y = torch.zeros((2, 100, 16), dtype=torch.complex64, device=dev)  # ldy = K: the plain detect, any R
    assert ofdm.zf_detect_pitched(Wt, Y).shape == (2, 4, 16)


@pytest.mark.parametrize("U,R,K,n,ldx,ldy", [(16, 64, 1023, 40, 1024, 1024), (16, 64, 1023, 17, 1023, 1024),
                                             (24, 16, 130, 9, 144, 131), (4, 8, 2, 5, 16, 3)])
def test_zf_apply_pitched(ofdm, oracle, dev, U, R, K, n, ldx, ldy):
    """ofdm_zf_apply_ex on row-padded layouts: pads untouched (NaN sentinels),
    results at the apply's 1e-5 bound against the oracle and bit-identical to
    the unpadded apply (the same 16-B-lane W-stationary kernel)."""
    import torch
    H = channel(U, R, K, seed=n + 9)
    W = oracle.zf_precoder(H)
    X = qpsk(n, U, K, seed=n + 10)
    ref = oracle.zf_apply(W, X)
    Wt = ofdm.zf_transpose(dev_t(W, dev))
    Xp = torch.full((n, U, ldx), float("nan"), dtype=torch.complex64, device=dev)
    Xp[:, :, :K] = dev_t(X, dev)
    out = torch.full((n, R, ldy), float("nan"), dtype=torch.complex64, device=dev)
    ofdm.zf_apply_pitched(Wt, Xp, out=out)
    got = out.cpu().numpy()
    assert np.isnan(got[:, :, K:]).all()
    parity(got[:, :, :K], ref)
    assert np.array_equal(got[:, :, :K], ofdm.zf_apply(Wt, dev_t(X, dev)).cpu().numpy())
