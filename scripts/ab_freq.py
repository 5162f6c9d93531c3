"""Same-process A/B of the frequency-domain combine: elementwise k_mrc_freq
vs the matrix-core k_mrc_freq_mfma (OFDM_MRC_FREQ_MFMA), BASELINE configs[4]'s
"compare MFMA-cgemm vs elementwise combine".  Times ofdm_frame_demod_freq
(LS + MRC on FFT'd symbols) with HIP events.
usage: python scripts/ab_freq.py [frames] [R] [C]"""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
import ofdm_lsmrc as ofdm

F = int(sys.argv[1]) if len(sys.argv) > 1 else 400
R = int(sys.argv[2]) if len(sys.argv) > 2 else 32
C = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
S, K = 101, C - 1
dev = torch.device("cuda")
rng = np.random.default_rng(1)
a = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)).to(dev)
Y = ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01, freq_domain=True)
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, K), dev)
res = {}
for rep in range(3):
    for v in ("0", "1"):
        os.environ["OFDM_MRC_FREQ_MFMA"] = v
        ofdm.frame_demod_freq(Y, X, ws, out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ofdm.frame_demod_freq(Y, X, ws, out)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(v, []).append(e0.elapsed_time(e1) / 5)
        if rep == 0:
            err = int(ofdm.count_symbol_errors(out, S, seed=1).item())
            print(f"MFMA={v}: {err} symbol errors")
Q = F * (S - 1)
b = Q * (R * C * 8 + K * 8) + F * R * C * 8
for v in ("0", "1"):
    ms = min(res[v])
    print(f"{'mfma' if v == '1' else 'elementwise':12s} R={R} C={C}: {ms:7.3f} ms  {Q / ms / 1e3:7.3f} M symbols/s  "
          f"{b / ms / 1e6:6.0f} GB/s  frac {b / ms / 1e6 / 8000:.3f}")
