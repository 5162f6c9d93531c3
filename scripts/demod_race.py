#!/usr/bin/env python3
"""Diagnostic for the one-launch frame demod (A/B build): repeated runs of
the normal path and the forced-fallback path (OFDM_AB_DEMOD_SPIN=0) against
the two-launch flow; prints, per trial, the max relative error and the
frames / symbols that differ.
usage: python scripts/demod_race.py [C] [frames] [trials] [R]"""
import os
import sys

os.environ.setdefault("OFDM_LSMRC_LIB", "ab")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402

arg = [int(x) for x in sys.argv[1:]] + [0] * 4
C = arg[0] or 1024
F, S, R = arg[1] or 9, 13, arg[3] or 16
trials = arg[2] or 4
a = np.float32(0.70710678)
rng = np.random.default_rng(5)
X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)).cuda()
iq = ofdm.synth_frames(F, S, R, C, X, seed=11, noise_std=0.01)
ws2 = ofdm.workspace(F, S, R, C, iq.device)
out2 = ofdm.c64((F, S - 1, C - 1), iq.device)
ofdm.frame_estimate(iq, X, 0, ws2)
ofdm.frame_combine(iq, 0, ws2, out2)
ref = out2.cpu().numpy()
scale = np.abs(ref).max()


def report(name, got):
    d = np.abs(got - ref) / scale
    bad = np.argwhere(d.max(axis=2) > 1e-5)
    print(f"C={C} {name}", "maxrel %.3g" % d.max(), "bad (frame, symbol):", bad[:12].tolist(), len(bad), flush=True)
    return d.max()


ws = ofdm.workspace(F, S, R, C, iq.device)
worst = 0.0
for trial in range(trials):
    os.environ.pop("OFDM_AB_DEMOD_SPIN", None)
    worst = max(worst, report(f"t{trial} normal", ofdm.frame_demod(iq, X, ws=ws).cpu().numpy()))
    os.environ["OFDM_AB_DEMOD_SPIN"] = "0"
    worst = max(worst, report(f"t{trial} spin0 ", ofdm.frame_demod(iq, X, ws=ws).cpu().numpy()))
os.environ.pop("OFDM_AB_DEMOD_SPIN", None)
sys.exit(0 if worst <= 1e-5 else 1)
