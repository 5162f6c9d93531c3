#!/usr/bin/env python3
"""Where does an A/B variant differ from the default kernel?  Prints the
(frame, symbol, bin) positions whose outputs differ by more than 1e-4."""
import os
import sys

os.environ["OFDM_LSMRC_LIB"] = "ab"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402

C = int(sys.argv[1])
knob = sys.argv[2]
S = 101
dev = torch.device("cuda")
for R, F in [(64, 8), (64, 400), (32, 40), (16, 40)]:
    K = C - 1
    rng = np.random.default_rng(1)
    amp = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-amp, amp], K) + 1j * rng.choice([-amp, amp], K)).astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01)
    ws = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_estimate(iq, X, 0, ws)
    outs = []
    for v in ["", knob]:
        os.environ.pop("OFDM_AB_" + knob.split("=")[0], None)
        if v:
            k, val = v.split("=")
            os.environ["OFDM_AB_" + k] = val
        out = ofdm.c64((F, S - 1, K), dev)
        ofdm.frame_combine(iq, 0, ws, out)
        torch.cuda.synchronize()
        outs.append(out)
    d = (outs[0] - outs[1]).abs()
    bad = (d > 1e-4).nonzero()
    print(f"R={R} F={F}: max {d.max().item():.3e}, {bad.shape[0]} positions > 1e-4", flush=True)
    for p in bad[:12].tolist():
        print("   ", p, outs[0][tuple(p)].item(), outs[1][tuple(p)].item(), flush=True)
    del iq, ws, outs
    torch.cuda.empty_cache()
