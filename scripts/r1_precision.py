#!/usr/bin/env python3
"""A/B build: parity metrics of the R = 1 receiver (single-antenna rows
amplify FFT rounding at deep-fade pilot bins) against the oracle, for the
kernel variants named on the command line (NAME=VAL switches, as ab.py)."""
import os
import sys

os.environ.setdefault("OFDM_LSMRC_LIB", "ab")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402
from oracle_bindings import Oracle  # noqa: E402
from test_gpu_parity import qpsk_pilots  # noqa: E402

o = Oracle()
dev = torch.device("cuda")
for C in (2048, 4096):
    F, S, R, prefix = 2, 6, 1, 0
    Xh = qpsk_pilots(C - 1)
    X = torch.from_numpy(Xh).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=99 + C, noise_std=0.05)
    ref = o.frames_demod(iq.cpu().numpy(), Xh, prefix, nthreads=8).astype(np.complex128).ravel()
    rms = np.sqrt(np.mean(np.abs(ref) ** 2))
    # what an f32 FFT (FFTW single precision in cpuLS) scores against the same f64 oracle
    r32 = o.frames_demod_fft32(iq.cpu().numpy(), Xh, prefix, nthreads=8).astype(np.complex128).ravel()
    e32 = np.abs(r32 - ref) / np.maximum(np.abs(ref), rms)
    print(f"C={C} {'oracle-f32':14s} norm-rel {np.linalg.norm(r32 - ref) / np.linalg.norm(ref):.3e} "
          f"elem-rel max {e32.max():.3e} 2nd {np.sort(e32)[-2]:.3e} p99 {np.percentile(e32, 99):.3e}", flush=True)
    for v in ["default"] + sys.argv[1:]:
        for kv in (v.split(",") if v != "default" else []):
            k, val = kv.split("=")
            os.environ["OFDM_AB_" + k] = val
        got = ofdm.frame_demod(iq, X, prefix).cpu().numpy().astype(np.complex128).ravel()
        for kv in (v.split(",") if v != "default" else []):
            del os.environ["OFDM_AB_" + kv.split("=")[0]]
        e = np.abs(got - ref) / np.maximum(np.abs(ref), rms)
        print(f"C={C} {v:14s} norm-rel {np.linalg.norm(got - ref) / np.linalg.norm(ref):.3e} "
              f"elem-rel max {e.max():.3e} 2nd {np.sort(e)[-2]:.3e} p99 {np.percentile(e, 99):.3e}", flush=True)
