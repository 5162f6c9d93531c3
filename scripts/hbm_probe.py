"""Diagnostic: achievable streaming-read bandwidth on this GPU (torch sum over
a large buffer) -- the practical ceiling the MRC kernel is compared with."""
import sys
import time
import torch
n_gb = float(sys.argv[1]) if len(sys.argv) > 1 else 32
x = torch.ones(int(n_gb * 2**30 / 4), dtype=torch.float32, device="cuda")
for _ in range(2):
    x.sum()
torch.cuda.synchronize()
t = time.perf_counter()
N = 5
for _ in range(N):
    x.sum()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / N
print(f"torch sum read: {x.numel() * 4 / dt / 1e9:.0f} GB/s over {n_gb} GiB")
y = torch.empty_like(x[: x.numel() // 2])
z = x[: x.numel() // 2]
for _ in range(2):
    y.copy_(z)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(N):
    y.copy_(z)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / N
print(f"torch copy: {2 * z.numel() * 4 / dt / 1e9:.0f} GB/s (read+write) over {n_gb / 2} GiB")
