"""Shared test helpers: fixture loading and the parity metric."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# north_star: "Results must match cpuLS.hpp on identical IQ input within 1e-5
# relative on complex<float>".  Checked two ways:
#   norm-relative   ||got - ref|| / ||ref||                      <= 1e-5
#   element-wise    |got - ref| <= 1e-5 * max(|ref|, rms(ref))   (rms floor
#                   for the rare near-zero outputs of a deep channel fade)
RTOL = 1e-5


def parity(got, ref, rtol=RTOL, erel_tol=None):
    got = np.asarray(got, np.complex128).ravel()
    ref = np.asarray(ref, np.complex128).ravel()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    if ref.size == 0:
        return 0.0, 0.0
    assert np.all(np.isfinite(got)), "non-finite output"
    nrel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
    rms = np.sqrt(np.mean(np.abs(ref) ** 2))
    erel = np.max(np.abs(got - ref) / np.maximum(np.abs(ref), rms))
    assert nrel <= rtol, f"norm-relative error {nrel:.3e} > {rtol:g}"
    etol = rtol if erel_tol is None else erel_tol
    assert erel <= etol, f"element-wise relative error {erel:.3e} > {etol:g}"
    return nrel, erel


def golden_cases(domain=None):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        z = np.load(p, allow_pickle=False)
        if domain is None or str(z["domain"]) == domain:
            out.append((os.path.basename(p)[:-4], z))
    return out
