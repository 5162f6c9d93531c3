#!/usr/bin/env python3
"""Same-process A/B of MRC kernel candidates in the A/B build
(make -C gpu-accel-ofdm-ls-mrc_amd ab -> lib/libofdm_lsmrc_ab.so, switches
OFDM_AB_<NAME> re-read per launch), so box-to-box clock and HBM variation do
not enter the comparison.  Variants are interleaved over repetitions.

usage: python scripts/ab.py [--C 1024] [--R 64] [--frames 400] [--reps 3] \
           default NAME=VAL[,NAME=VAL...] ...
Prints one JSON line per variant: ms per frame_combine launch (median over
reps of the mean of 5 launches), algorithmic TB/s (R*C*8 + K*8 per data
symbol) and fraction of 8 TB/s, QPSK errors, max |difference| vs the first
variant.  Variants whose name contains DBG are diagnostics (wrong results by
design): no error/equality checks.
"""
import argparse
import json
import os
import sys

os.environ.setdefault("OFDM_LSMRC_LIB", "ab")  # or another non-product build (scripts/libab.py)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--C", type=int, default=1024)
ap.add_argument("--R", type=int, default=64)
ap.add_argument("--S", type=int, default=101)
ap.add_argument("--frames", type=int, default=400)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--partial", action="store_true", help="time frame_mrc_partial (numerators)")
ap.add_argument("--ls", action="store_true", help="time frame_estimate (the LS kernel) instead of the MRC")
ap.add_argument("--demod", action="store_true",
                help="time frame_demod (LS + MRC: one launch at C = 1024 / 2048 / 4096 unless DEMOD_FUSED=0)")
ap.add_argument("--freq", action="store_true",
                help="frequency-domain frames: time frame_demod_freq (LS + MRC, no FFT)")
ap.add_argument("--allocs", type=int, default=1,
                help="repeat the comparison on N separately allocated copies of the batch (what the "
                     "output stores cost depends on where the input lives: DESIGN.md 4.3)")
ap.add_argument("--ls-per-variant", action="store_true",
                help="re-run the LS estimate under each variant's switches (variants that change the Hc layout)")
ap.add_argument("variants", nargs="*", default=["default"])
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402

assert not ofdm.LIB_PATH.endswith("libofdm_lsmrc.so") or os.environ["OFDM_LSMRC_LIB"] == "", ofdm.LIB_PATH
F, S, R, C = a.frames, a.S, a.R, a.C
K = C - 1
Q = F * (S - 1)
dev = torch.device("cuda")
rng = np.random.default_rng(1)
amp = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-amp, amp], K) + 1j * rng.choice([-amp, amp], K))
                     .astype(np.complex64)).to(dev)
iqs = [ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01, freq_domain=a.freq) for _ in range(a.allocs)]
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, K), dev)


def estimate():
    global ws
    if a.freq:
        pass
    elif a.partial:
        _, ws = ofdm.frame_ls_partial(iq, X, 0, ws=ws)
    else:
        ofdm.frame_estimate(iq, X, 0, ws)


keys = {kv.split("=")[0] for v in a.variants if v != "default" for kv in v.split(",")}


def run():
    if a.freq:
        ofdm.frame_demod_freq(iq, X, ws=ws, out=out)
        return
    if a.ls:
        ofdm.frame_estimate(iq, X, 0, ws)
        return
    if a.demod:
        ofdm.frame_demod(iq, X, 0, ws=ws, out=out)
        return
    if a.partial:
        ofdm.frame_mrc_partial(iq, ws, 0, num=out)
    else:
        ofdm.frame_combine(iq, 0, ws, out)


for ai, iq in enumerate(iqs):
    estimate()
    res = {v: [] for v in a.variants}
    chk = {}
    ref = None
    for rep in range(a.reps):
        for v in a.variants:
            for k in keys:
                os.environ.pop("OFDM_AB_" + k, None)
            if v != "default":
                for kv in v.split(","):
                    k, val = kv.split("=")
                    os.environ["OFDM_AB_" + k] = val
            if a.ls_per_variant:
                estimate()
            run()  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 5)
            if rep == 0 and "DBG" not in v:
                if a.ls:  # check the variant's estimate end to end
                    ofdm.frame_combine(iq, 0, ws, out)
                errs = None if a.partial else int(ofdm.count_symbol_errors(out, S, seed=1).item())
                if ref is None:
                    ref = out.clone()
                    d = 0.0
                else:
                    d = (out - ref).abs().max().item()
                chk[v] = (errs, d)
    b_sym = (R * C * 8 * 2 / (S - 1)) if a.ls else (R * C * 8 + K * 8)  # LS: pilot rows in + Hc out
    if a.demod:
        b_sym = R * C * 8 * S / (S - 1) + K * 8  # pilot + data rows in, outputs
    for v in a.variants:
        ms = sorted(res[v])[len(res[v]) // 2]
        tbs = Q * b_sym / (ms * 1e-3) / 1e12
        e, d = chk.get(v, (None, None))
        print(json.dumps({"variant": v, "C": C, "R": R, "frames": F, "ms": round(ms, 4),
                          "all_ms": [round(x, 4) for x in res[v]], "TBps": round(tbs, 3),
                          "frac_8TBps": round(tbs / 8.0, 4), "alloc": ai, "qpsk_errors": e, "max_abs_diff_vs_first": d}),
              flush=True)
