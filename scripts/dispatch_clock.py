#!/usr/bin/env python3
"""Per-dispatch clock and timeline of back-to-back one-launch steps
(k_demod_td1024), from the diagnostic build (lib/libofdm_lsmrc_diag.so: the
same kernel with per-workgroup s_memtime / s_memrealtime stamps, written
into slot (launch epoch mod 32) of its stamp buffer, csrc/diag.hpp).

Runs bench.py's frames-mode step with the DIAGNOSTIC library as the timed
one: W warm-up steps, an optional idle gap (bench.py's flow has one: the
warm-up check between warm-up and the timed loop), K timed steps with HIP
events per step; then reads the last min(K, 32) launches' stamps.  Prints
one JSON line per timed dispatch: event ms, stamped span, median effective
clock, estimator span, MRC start delay, tail (time from the active count's
fall below half its peak to the end), and a summary line.

usage: python scripts/dispatch_clock.py [--R 16] [--frames 100] [--steps 20]
                                        [--warmup 5] [--gap-ms 9]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ["OFDM_LSMRC_LIB"] = "diag"

ap = argparse.ArgumentParser()
ap.add_argument("--R", type=int, default=16)
ap.add_argument("--frames", type=int, default=100)
ap.add_argument("--S", type=int, default=101)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--gap-ms", type=float, default=0.0, help="idle time between warm-up and timed steps")
ap.add_argument("--tag", default="")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402
from wg_timeline import analyse  # noqa: E402

assert ofdm.LIB_PATH.endswith("libofdm_lsmrc_diag.so"), ofdm.LIB_PATH
L = ofdm.lib()
read, clear = L.ofdm_diag_read_td1024, L.ofdm_diag_clear_td1024
read.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
F, S, R, C = a.frames, a.S, a.R, 1024
K = C - 1
dev = torch.device("cuda")
rng = np.random.default_rng(1234)
amp = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-amp, amp], K) + 1j * rng.choice([-amp, amp], K)).astype(np.complex64)).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, seed=1234, noise_std=0.01)
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, K), dev)
stream = torch.cuda.current_stream()
nls = (F + 7) // 8 * 8
for _ in range(a.warmup):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=stream)
torch.cuda.synchronize()
clear()
torch.cuda.synchronize()
if a.gap_ms > 0:
    time.sleep(a.gap_ms * 1e-3)
evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
evs[0].record(stream)
for i in range(a.steps):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=stream)
    evs[i + 1].record(stream)
torch.cuda.synchronize()
ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)]
errs = int(ofdm.count_symbol_errors(out, S, seed=1234).item())
rec = np.zeros((1 << 20, 12), dtype=np.uint64)  # diag::WORDS
assert read(rec.ctypes.data, 1 << 20) == 0
slots = rec.reshape(32, -1, 12)
runs = []
for sl in slots:
    r = sl[sl[:, 2] > 0]
    if len(r):
        # only the slot's latest launch (word 7's high half = launch counter)
        r = r[(r[:, 7] >> 32) == (r[:, 7] >> 32).max()]
        r[:, 7] &= 0xFFFFFFFF
        runs.append((int(r[:, 0].min()), r))
runs.sort(key=lambda x: x[0])
# the last len(runs) timed dispatches, in order
ms_tail = ms[-len(runs):]
base = runs[0][0]
rows = []
for i, ((t0, r), m) in enumerate(zip(runs, ms_tail)):
    an = analyse(r, nls)
    est, mrc = an.get("estimator", {}), an.get("mrc", {})
    row = {"tag": a.tag, "dispatch": a.steps - len(runs) + i, "event_ms": m, "start_ms": (t0 - base) * 1e-5,
           "span_us": an["span_us"], "GHz_mrc": mrc.get("GHz_median"), "GHz_est": est.get("GHz_median"),
           "est_end_us_p50_p100": [est["end_us"][2], est["end_us"][4]] if est else None,
           "mrc_wait_us_p50_p90": [mrc["mark_minus_start_us"][2], mrc["mark_minus_start_us"][3]] if mrc else None,
           "mrc_life_us_p50": mrc["life_us"][2] if mrc else None,
           "tail_us": an["tail_us_below_half_peak"], "ramp_us": an["ramp_us_to_90pct"],
           "active_peak": an["active_peak"], "occupancy_fill": an["occupancy_fill"]}
    rows.append(row)
    print(json.dumps(row), flush=True)
print(json.dumps({"tag": a.tag, "summary": True, "R": R, "frames": F, "steps": a.steps, "warmup": a.warmup,
                  "gap_ms": a.gap_ms, "mean_ms": sum(ms) / len(ms), "first5_ms": ms[:5], "last5_ms": ms[-5:],
                  "qpsk_errors": errs,
                  "GHz_first_last": [rows[0]["GHz_mrc"], rows[-1]["GHz_mrc"]] if rows else None}), flush=True)
