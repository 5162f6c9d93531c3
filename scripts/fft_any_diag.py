"""Phase timing of k_fft_any (diagnostic build with s_memtime stamps and a
printf per 97th workgroup; OFDM_LSMRC_LIB=diag): cycles per row group spent
waiting for the prefetched rows + writing them to LDS, in the stages, in the
global stores and at the closing barrier."""
import sys
import numpy as np
import torch
sys.path.insert(0, "gpu-accel-ofdm-ls-mrc_amd")
import ofdm_lsmrc as ofdm

C = int(sys.argv[1]) if len(sys.argv) > 1 else 1536
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 64 * 101 * 200
x = torch.randn(rows, C, dtype=torch.complex64, device="cuda")
out = torch.empty_like(x)
for _ in range(3):
    ofdm.fft_rows(x, out)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
ofdm.fft_rows(x, out)
ev[1].record()
torch.cuda.synchronize()
ms = ev[0].elapsed_time(ev[1])
print(f"C={C} rows={rows} {ms:.3f} ms  {rows * C * 16 / ms / 1e9:.2f} TB/s (read + write)", flush=True)
