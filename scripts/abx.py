#!/usr/bin/env python3
"""Same-process A/B of whole library builds: the product library and variants
built by scripts/build_variant.sh (lib/libofdm_lsmrc_<name>.so) are loaded
side by side in ONE process and called alternately on the same device-resident
batch, so clock and HBM differences between boxes and runs do not enter the
comparison.  No experiment switch lives in the product sources.

usage: python scripts/abx.py [--C 4096] [--R 32] [--frames 300] [--reps 3]
                             [--stage demod|combine|partial] prod base [name ...]
One JSON line per (library, rep) and a summary per library: ms per launch
(mean of --launches launches, HIP events on the launch stream), algorithmic
TB/s (R*C*8 + K*8 per data symbol; + the pilot symbol per frame for demod),
QPSK errors, max |difference| vs the first library.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--C", type=int, default=4096)
ap.add_argument("--R", type=int, default=32)
ap.add_argument("--S", type=int, default=101)
ap.add_argument("--frames", type=int, default=300)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--launches", type=int, default=5)
ap.add_argument("--stage", choices=["demod", "combine", "partial"], default="combine")
ap.add_argument("libs", nargs="+")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402


def load(name):
    path = ofdm.LIB_PATH if name == "prod" else os.path.join(ofdm.HERE, "lib", f"libofdm_lsmrc_{name}.so")
    L = ctypes.CDLL(path)
    for fn, (res, args) in ofdm._SIGS.items():
        if hasattr(L, fn):
            f = getattr(L, fn)
            f.restype, f.argtypes = res, args
    return L


ofdm.lib()
libs = {n: load(n) for n in a.libs}
F, S, R, C = a.frames, a.S, a.R, a.C
K = C - 1
Q = F * (S - 1)
dev = torch.device("cuda")
rng = np.random.default_rng(1)
amp = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-amp, amp], K) + 1j * rng.choice([-amp, amp], K)).astype(np.complex64)).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01)
ws = {}
for n in a.libs:  # each build sizes its own workspace (ofdm_frame_workspace_bytes)
    ofdm._lib = libs[n]
    ws[n] = ofdm.workspace(F, S, R, C, dev)
ofdm._lib = libs[a.libs[0]]
out = {n: ofdm.c64((F, S - 1, K), dev) for n in a.libs}
stream = torch.cuda.current_stream()
b_sym = R * C * 8 + K * 8
nbytes = Q * b_sym + (F * (R * C * 8 + K * 8) if a.stage == "demod" else 0)


def run(n):
    ofdm._lib = libs[n]
    if a.stage == "demod":
        ofdm.frame_demod(iq, X, 0, ws=ws[n], out=out[n], stream=stream)
    elif a.stage == "combine":
        ofdm.frame_combine(iq, 0, ws[n], out[n], stream)
    else:
        ofdm.frame_mrc_partial(iq, ws[n], 0, num=out[n], stream=stream)


for n in a.libs:  # estimates + warm-up
    ofdm._lib = libs[n]
    if a.stage == "combine":
        ofdm.frame_estimate(iq, X, 0, ws[n], stream)
    elif a.stage == "partial":
        ofdm.frame_ls_partial(iq, X, 0, ws=ws[n], stream=stream)
    run(n)
torch.cuda.synchronize()
ref = out[a.libs[0]].clone()
res = {n: [] for n in a.libs}
for rep in range(a.reps):
    for n in (a.libs if rep % 2 == 0 else a.libs[::-1]):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(a.launches):
            run(n)
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.launches
        d = float((out[n] - ref).abs().max())
        errs = int(ofdm.count_symbol_errors(out[n], S, seed=1).item()) if a.stage != "partial" else None
        res[n].append(ms)
        print(json.dumps({"lib": n, "rep": rep, "stage": a.stage, "C": C, "R": R, "frames": F, "ms": ms,
                          "TBps": nbytes / ms / 1e9, "frac": nbytes / ms / 1e9 / 8.0, "max_diff_vs_first": d,
                          "bit_identical": d == 0.0, "qpsk_errors": errs}), flush=True)
for n, v in res.items():
    m = sorted(v)[len(v) // 2]
    print(f"{n}: median {m:.3f} ms = {nbytes / m / 1e9:.3f} TB/s ({nbytes / m / 8e9 * 100:.1f} % of 8 TB/s); "
          f"all {' '.join(f'{x:.3f}' for x in v)}", flush=True)
