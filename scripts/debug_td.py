"""Diagnostic: run the fused C=1024 estimate on one frame and compare the
workspace channel estimates (lane-ordered) with the oracle, per lane/bin."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"), os.path.join(ROOT, "tests")]
import ofdm_lsmrc as ofdm
from oracle_bindings import Oracle

F, S, R, C, pre = 1, 3, 4, 1024, 0
dev = torch.device("cuda")
rng = np.random.default_rng(0)
Xh = ((rng.choice([-1, 1], C - 1) + 1j * rng.choice([-1, 1], C - 1)) * 0.70710678).astype(np.complex64)
X = torch.from_numpy(Xh).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, prefix=pre, seed=3, noise_std=0.01)
ws = ofdm.workspace(F, S, R, C, dev)
ofdm.frame_estimate(iq, X, pre, ws)
torch.cuda.synchronize()
wsh = ws.cpu().numpy()
Hl = wsh[: F * R * C * 8].view(np.complex64).reshape(F, R, 8, 64, 2)  # [f][r][i][t][2]
P = wsh[((F * R * C * 8 + 255) // 256) * 256:][: F * C * 4].view(np.float32).reshape(F, C)
o = Oracle()
_, Href, Pref = o.frame_demod(iq[0].cpu().numpy(), Xh, pre)
t = np.arange(64)
b0 = (t >> 2) + 256 * (((t & 3) >> 1) + 2 * (t & 1))
bad_lanes = set()
for r in range(R):
    for tt in t:
        for k in range(16):
            b = b0[tt] + 16 * k
            h = Hl[0, r, k // 2, tt, k % 2]
            ref = 0 if b == 0 else Href[r, b - 1]
            if abs(h - ref) > 1e-3 * (abs(ref) + 1e-3):
                bad_lanes.add(int(tt))
print("bad lanes (Hc):", sorted(bad_lanes)[:64], "count", len(bad_lanes))
pb = np.abs(P[0, 1:] - Pref) > 1e-3 * np.abs(Pref)
print("P bad bins:", np.nonzero(pb)[0][:20], pb.sum())
out = ofdm.c64((F, S - 1, C - 1), dev)
ofdm.frame_combine(iq, pre, ws, out)
ref = o.frames_demod(iq.cpu().numpy(), Xh, pre)
d = np.abs(out.cpu().numpy() - ref)
print("out max err", d.max(), "bad", (d > 1e-4).sum(), "of", d.size)
