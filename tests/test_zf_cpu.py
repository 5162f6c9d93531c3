"""Zero-forcing oracle (oracle/zf_oracle.c, restating createZeroForcingMatrix /
multiplyWithChannelInv, cpuLS.hpp:400-463) pinned on the CPU.

The reference computes these with CBLAS (cgemm, cgemv) and LAPACK (cgetrf,
cgetri), none of which is installed here, and has no tests or fixtures for
them.  Parity is pinned by
  * the reference's own rotCube (compiled from /root/reference by
    oracle/build_ref.sh), which fixes how the channel cube is read: the
    per-subcarrier A handed to cgemm, and W's output layout (ldc = rows);
  * an independent float64 numpy restatement (numpy's LAPACK inverse) of the
    cgemm / cgetrf+cgetri / cgemm sequence, within f32 rounding.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle_bindings import reference_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd")


def build_zf_driver(tmp):
    """tests/cpp/zf_driver.cpp against the drop-in cpuLS.hpp + the library."""
    exe = os.path.join(tmp, "zf_driver")
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{PKG}/host", f"-I{ROOT}/include", os.path.join(ROOT, "tests", "cpp", "zf_driver.cpp"),
                    "-o", exe, f"-L{PKG}/lib", "-lofdm_lsmrc", f"-Wl,-rpath,{PKG}/lib",
                    "-L/opt/rocm/lib", "-lamdhip64", "-lrt"], check=True)
    return exe


def test_cpuls_zf_api_compiles_and_links(tmp_path):
    """The reference's ZF call sequence compiles against the drop-in
    cpuLS.hpp and links against the library (run on the GPU in test_zf_gpu)."""
    if not os.path.exists(os.path.join(PKG, "lib", "libofdm_lsmrc.so")):
        pytest.skip("library not built")
    assert os.path.exists(build_zf_driver(str(tmp_path)))
from zf_cases import channel, qpsk, rel_err, rel_err_per_subcarrier, zf_numpy

SHAPES = [(1, 1, 3), (2, 4, 7), (4, 16, 31), (8, 64, 15), (16, 64, 9), (32, 64, 5), (3, 5, 4),
          (16, 512, 3)]


@pytest.mark.parametrize("U,R,K", SHAPES)
def test_oracle_precoder_matches_float64(oracle, U, R, K):
    H = channel(U, R, K, seed=U * 1000 + R + K)
    W = oracle.zf_precoder(H)
    assert W.shape == (K, U, R)
    # tolerance: f32 LU + inverse of G = A A^H, cond(G) = cond(A)^2 (< ~1e3 here)
    assert rel_err_per_subcarrier(W, zf_numpy(H)) < 2e-4


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built (no /root/reference)")
def test_rotcube_layout_pins_oracle(oracle):
    """Drive the per-subcarrier BLAS calls of createZeroForcingMatrix
    (cpuLS.hpp:436-441) on the buffer the reference's own rotCube produces,
    with numpy standing in for cgemm / cgetrf+cgetri, and compare with the
    oracle's W in the reference's H layout."""
    from oracle_bindings import Reference
    ref = Reference()
    U, R, K = 4, 8, 11
    H = channel(U, R, K, seed=5)
    Xr = ref.rot_cube(H)  # reference rotCube(X, rows, cols=K, users)
    W = oracle.zf_precoder(H)
    for col in range(K):
        blk = Xr[col * R * U:(col + 1) * R * U].astype(np.complex128)
        A = blk.reshape(R, U).T  # column-major users x rows, lda = users
        assert np.array_equal(A.astype(np.complex64), H[:, :, col])
        G = A @ A.conj().T  # cgemm(NoTrans, ConjTrans, users, users, rows)
        Wk = A.conj().T @ np.linalg.inv(G)  # cgemm(ConjTrans, NoTrans, rows, users, users)
        out = Wk.T.ravel()  # column-major rows x users, ldc = rows: element (r, u) at r + u*rows
        assert rel_err(W[col].ravel(), out) < 1e-5


@pytest.mark.parametrize("U,R,K,n", [(1, 1, 3, 1), (4, 16, 31, 3), (16, 64, 9, 2), (3, 5, 4, 5)])
def test_oracle_apply_detect_match_float64(oracle, U, R, K, n):
    H = channel(U, R, K, seed=7)
    W = oracle.zf_precoder(H)
    X = qpsk(n, U, K)
    Y = oracle.zf_apply(W, X)
    W64 = W.astype(np.complex128)
    assert rel_err(Y, np.einsum("kur,suk->srk", W64, X)) < 1e-6
    Xh = oracle.zf_detect(W, Y)
    assert rel_err(Xh, np.einsum("kur,srk->suk", W64.conj(), Y.astype(np.complex128))) < 1e-6


def test_oracle_zero_forcing_round_trips(oracle):
    """The defining property: the precoded downlink through the channel and
    ZF detection of the uplink both return the users' symbols."""
    U, R, K, n = 8, 32, 17, 4
    H = channel(U, R, K, seed=11)
    W = oracle.zf_precoder(H)
    X = qpsk(n, U, K)
    Hd = H.astype(np.complex128)
    down = np.einsum("urk,srk->suk", Hd, oracle.zf_apply(W, X).astype(np.complex128))
    assert rel_err(down, X) < 1e-4
    up = np.einsum("urk,suk->srk", Hd.conj(), X.astype(np.complex128)).astype(np.complex64)
    assert rel_err(oracle.zf_detect(W, up), X) < 1e-4
