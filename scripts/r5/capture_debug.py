# debug: graph capture of the ticketed C = 4096 receiver; NaN units after one replay, counters
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gpu-accel-ofdm-ls-mrc_amd"))
import numpy as np, torch
import ofdm_lsmrc as ofdm
C, F, R, S = 4096, 16, 4, 101
dev = torch.device("cuda")
rng = np.random.default_rng(1)
a = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, seed=5, noise_std=0.01)
ref = ofdm.frame_demod(iq, X, 0)
ws = ofdm.workspace(F, S, R, C, dev)
out = ofdm.c64((F, S - 1, C - 1), dev)
st = torch.cuda.Stream()
ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
torch.cuda.synchronize()
print("eager equal", torch.equal(out, ref))
up = lambda n: (n + 255) // 256 * 256
off = up(F * R * C * 8) + up(F * C * 4) + up(F * 8)
wsb = ws.view(torch.uint8) if ws.dtype != torch.uint8 else ws
def counters():
    t = wsb[off:off + 4096].clone().view(torch.int64).cpu().numpy()
    return [t[s * 128:(s + 1) * 128:16].tolist() for s in range(4)]
print("ws dtype", ws.dtype, ws.numel(), "counters after eager", counters())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
for rep in range(3):
    out.fill_(float("nan"))
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    nan = torch.isnan(out.real).any(dim=2).cpu().numpy()  # [F][S-1]
    print("replay", rep, "equal", torch.equal(out, ref), "nan symbols", int(nan.sum()), "first", np.argwhere(nan)[:5].tolist(), "counters", counters())
