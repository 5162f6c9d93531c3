#!/usr/bin/env python3
"""A/B build only: check the register-only 1024-point FFT (csrc/rfft1024.hpp)
against numpy, then time it against the receiver's LDS-transpose FFT in a
compute-only loop (csrc/rfft_test.hip), at 2 and 4 waves per SIMD."""
import ctypes as C
import json
import os
import sys

os.environ["OFDM_LSMRC_LIB"] = "ab"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402

L = ofdm.lib()
dev = torch.device("cuda")
rng = np.random.default_rng(5)
n = 256
x = (rng.standard_normal((n, 1024)) + 1j * rng.standard_normal((n, 1024))).astype(np.complex64)
xi = torch.from_numpy(x).to(dev)
xo = torch.empty_like(xi)
f = L.ofdm_ab_rfft_check
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
assert f(xi.data_ptr(), xo.data_ptr(), n, None) == 0
torch.cuda.synchronize()
ref = np.fft.fft(x.astype(np.complex128), axis=1)
got = xo.cpu().numpy()
err = np.abs(got - ref).max() / np.abs(ref).max()
print(json.dumps({"check": "rfft1024 vs numpy", "rows": n, "max_rel_err": float(err)}), flush=True)
if err > 1e-5:
    # diagnose: for each output slot, the reference bin whose column it matches best
    g = got / np.linalg.norm(got, axis=0, keepdims=True).clip(1e-30)
    r = ref / np.linalg.norm(ref, axis=0, keepdims=True)
    corr = np.abs(g.conj().T @ r)  # [slot][bin]
    best = corr.argmax(axis=1)
    print(json.dumps({"slots_matching_own_bin": int((best == np.arange(1024)).sum()),
                      "best_corr_min": float(corr.max(axis=1).min()),
                      "first_slots": [[int(p), int(best[p]), round(float(corr[p, best[p]]), 3)]
                                      for p in range(0, 1024, 37)]}), flush=True)
    sys.exit(1)

b = L.ofdm_ab_fft_bench
b.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_int, C.c_void_p]
nblocks = 256 * 8
rows = nblocks * 8
bi = torch.randn(rows, 1024, dtype=torch.complex64, device=dev)
bo = torch.empty_like(bi)
iters = 64
names = {0: "lds_transpose", 2: "lds_transpose_pk", 1: "register_only"}
for wpe in (2, 4):
    res = {}
    for rep in range(3):
        for v in (0, 2, 1):
            assert b(bi.data_ptr(), bo.data_ptr(), nblocks, iters, v, wpe, None) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert b(bi.data_ptr(), bo.data_ptr(), nblocks, iters, v, wpe, None) == 0
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(v, []).append(e0.elapsed_time(e1))
    for v in (0, 2, 1):
        ms = sorted(res[v])[1]
        print(json.dumps({"variant": names[v], "waves_per_simd": wpe, "ms": round(ms, 4),
                          "ns_per_fft": round(ms * 1e6 / (rows * iters), 4)}), flush=True)
