# where the one-launch and two-launch flows differ most at R = 1 (many frames): the worst
# elements' |ref| / rms (deep fades make |Y / H| large) and the oracle's float64 answer there
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gpu-accel-ofdm-ls-mrc_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests")]
import numpy as np, torch
import ofdm_lsmrc as ofdm
from oracle_bindings import Oracle
C, F, S, R = 1024, 20000, 3, 1
dev = torch.device("cuda")
rng = np.random.default_rng(C + F)
a = np.float32(0.70710678)
X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)).to(dev)
iq = ofdm.synth_frames(F, S, R, C, X, seed=F, noise_std=0.01)
one = ofdm.frame_demod(iq, X, 0).cpu().numpy().ravel()
ws = ofdm.workspace(F, S, R, C, dev); out2 = ofdm.c64((F, S - 1, C - 1), dev)
ofdm.frame_estimate(iq, X, 0, ws); ofdm.frame_combine(iq, 0, ws, out2)
two = out2.cpu().numpy().ravel()
rms = np.sqrt(np.mean(np.abs(two) ** 2))
err = np.abs(one - two) / np.maximum(np.abs(two), rms)
idx = np.argsort(err)[-5:]
print("max erel", err.max(), "elements > 1e-5:", int((err > 1e-5).sum()), "of", err.size)
print("worst |ref|/rms:", (np.abs(two[idx]) / rms).round(1).tolist())
# oracle (float64 FFT) on the frames holding the worst elements
o = Oracle()
fr = sorted(set((idx // ((S - 1) * (C - 1))).tolist()))
ref = o.frames_demod(iq[fr].cpu().numpy(), X.cpu().numpy(), 0)
for i in idx:
    f = i // ((S - 1) * (C - 1)); k = i % ((S - 1) * (C - 1))
    r = ref[fr.index(f)].ravel()[k]
    print(f"frame {f}: one-launch err vs oracle {abs(one[i]-r)/abs(r):.2e}, two-launch {abs(two[i]-r)/abs(r):.2e}")
