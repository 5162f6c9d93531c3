#!/usr/bin/env python3
"""BASELINE configs[4]'s comparison: the antenna combine as MFMA-cgemm
(ofdm_frame_demod_freq_mfma, mrc_mfma.hip) vs elementwise (ofdm_frame_demod_freq,
k_mrc_freq_frames) on the same frequency-domain frames, interleaved in one
process.  Run it under `rocprofv3 --kernel-trace --stats` for per-kernel times.

usage: python scripts/ab_mfma.py [frames] [R] [C] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402

F, R, C = (int(v) for v in (sys.argv[1:4] + ["400", "32", "4096"][len(sys.argv[1:4]):]))
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 9
S, K = 101, C - 1
Q = F * (S - 1)
dev = torch.device("cuda")
rng = np.random.default_rng(3)
a = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)).to(dev)
Y = ofdm.synth_frames(F, S, R, C, X, seed=3, noise_std=0.01, freq_domain=True)
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, K), dev)
fns = {"elementwise": lambda: ofdm.frame_demod_freq(Y, X, ws=ws, out=out),
       "mfma": lambda: ofdm.frame_demod_freq_mfma(Y, X, ws=ws, out=out)}
res = {k: [] for k in fns}
errs, outs = {}, {}
for rep in range(reps):
    for k, fn in fns.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1))
        if rep == 0:
            errs[k] = int(ofdm.count_symbol_errors(out, S, seed=3).item())
            outs[k] = out.clone()
diff = (outs["mfma"] - outs["elementwise"]).abs().max().item()
for k, v in res.items():
    ms = sorted(v)[len(v) // 2]
    tbs = Q * (R * C * 8 + K * 8) / (ms * 1e-3) / 1e12
    print(json.dumps({"combine": k, "R": R, "C": C, "frames": F, "ms_ls_plus_mrc": round(ms, 4),
                      "symbols_per_s": round(Q / (ms * 1e-3)), "TBps": round(tbs, 3),
                      "frac_8TBps": round(tbs / 8, 4), "qpsk_errors": errs[k],
                      "max_abs_diff_mfma_vs_elementwise": diff}), flush=True)
