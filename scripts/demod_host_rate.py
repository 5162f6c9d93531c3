"""Host enqueue rate vs GPU time of back-to-back ofdm_frame_demod calls
(configs[1] by default): is the one-launch loop host-bound?"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-accel-ofdm-ls-mrc_amd"))
import ofdm_lsmrc as ofdm

F, S, R, C = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (100, 101, 16, 1024)))
K = int(sys.argv[5]) if len(sys.argv) > 5 else 200
dev = torch.device("cuda:0")
rng = np.random.default_rng(5)
a = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01)
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, C - 1), dev)
st = torch.cuda.Stream()
for _ in range(20):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
# host-only: calls enqueued with the GPU held busy by nothing
t0 = time.perf_counter()
e0.record(st)
for _ in range(K):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
t1 = time.perf_counter()
e1.record(st)
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"F={F} S={S} R={R} C={C} K={K}: host enqueue {1e6*(t1-t0)/K:.1f} us/call, "
      f"GPU {1e3*e0.elapsed_time(e1)/K:.1f} us/call, wall {1e6*(t2-t0)/K:.1f} us/call")
# the same with the launches queued behind a long GPU wait (host runs ahead)
torch.cuda._sleep(int(2e9)) if hasattr(torch.cuda, "_sleep") else None
t0 = time.perf_counter()
e0.record(st)
for _ in range(K):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
e1.record(st)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"queued behind sleep: host {1e6*(t1-t0)/K:.1f} us/call, GPU {1e3*e0.elapsed_time(e1)/K:.1f} us/call")
