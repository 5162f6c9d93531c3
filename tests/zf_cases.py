"""Seeded inputs for the zero-forcing tests (channel cubes in the layout the
reference hands to rotCube, cpuLS.hpp:400-413: H[user][row][subcarrier])."""
import numpy as np


def channel(U, R, K, seed=0):
    rng = np.random.default_rng(seed)
    s = np.sqrt(0.5)
    return ((rng.standard_normal((U, R, K)) + 1j * rng.standard_normal((U, R, K))) * s).astype(
        np.complex64)


def qpsk(n, U, K, seed=1):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 2, size=(2, n, U, K))
    a = np.float32(np.sqrt(0.5))
    return ((2 * b[0] - 1) * a + 1j * (2 * b[1] - 1) * a).astype(np.complex64)


def zf_numpy(H):
    """float64 W[k][u][r] = (A^H (A A^H)^-1)(r, u), A(u, r) = H[u][r][k]."""
    U, R, K = H.shape
    W = np.empty((K, U, R), np.complex128)
    for k in range(K):
        A = H[:, :, k].astype(np.complex128)
        Wk = A.conj().T @ np.linalg.inv(A @ A.conj().T)  # R x U
        W[k] = Wk.T
    return W


def rel_err_per_subcarrier(got, ref):
    """max over subcarriers of ||got_k - ref_k|| / ||ref_k|| (W layout [K][U][R])."""
    got = got.astype(np.complex128).reshape(got.shape[0], -1)
    ref = ref.astype(np.complex128).reshape(ref.shape[0], -1)
    return float((np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)).max())


def rel_err(got, ref):
    got = got.astype(np.complex128)
    ref = ref.astype(np.complex128)
    return float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
