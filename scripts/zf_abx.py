#!/usr/bin/env python3
"""Same-process A/B of ZF detect / apply across whole library builds (the
product and lib/libofdm_lsmrc_<name>.so from scripts/build_variant.sh),
alternating per round on the same device-resident data.

usage: python scripts/zf_abx.py [--U 16] [--R 64] [--nsym 10000] prod NAME ...
One JSON line per (library, round); then per library the median detect /
apply ms, % of 8 TB/s ((U + R) * K * 8 B per symbol) and the max relative
difference from the first library's outputs."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"), os.path.join(ROOT, "tests")]
ap = argparse.ArgumentParser()
ap.add_argument("--U", type=int, default=16)
ap.add_argument("--R", type=int, default=64)
ap.add_argument("--K", type=int, default=1023)
ap.add_argument("--nsym", type=int, default=10000)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402
from zf_cases import channel  # noqa: E402

libs = {n: (ofdm.lib() if n == "prod" else ofdm.load_library(os.path.join(ofdm.HERE, "lib", f"libofdm_lsmrc_{n}.so")))
        for n in a.libs}
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(0)
U, R, K, n = a.U, a.R, a.K, a.nsym
Y = torch.randn((n, R, K), dtype=torch.complex64, device=dev, generator=g)
X = torch.randn((n, U, K), dtype=torch.complex64, device=dev, generator=g)
W, Wt = ofdm.zf_precoder(torch.from_numpy(channel(U, R, K, seed=U)).to(dev))
out = {nm: (torch.empty_like(X), torch.empty_like(Y)) for nm in a.libs}
nbytes = (U + R) * K * 8 * n


def timed(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps


res = {nm: [] for nm in a.libs}
for rnd in range(a.rounds):
    for nm in (a.libs if rnd % 2 == 0 else a.libs[::-1]):
        Xo, Yo = out[nm]
        with ofdm.using(libs[nm]):
            d = timed(lambda: ofdm.zf_detect(Wt, Y, out=Xo))
            p = timed(lambda: ofdm.zf_apply(Wt, X, out=Yo))
        res[nm].append((d, p))
        print(json.dumps({"lib": nm, "round": rnd, "U": U, "R": R, "nsym": n, "detect_ms": d, "apply_ms": p}),
              flush=True)
ref = out[a.libs[0]]
for nm, v in res.items():
    d = sorted(x[0] for x in v)[len(v) // 2]
    p = sorted(x[1] for x in v)[len(v) // 2]
    dx = float(((out[nm][0] - ref[0]).abs().max() / ref[0].abs().max()).item())
    dy = float(((out[nm][1] - ref[1]).abs().max() / ref[1].abs().max()).item())
    print(f"{nm}: detect {d:.3f} ms = {nbytes / d / 8e9 * 100:.1f} %, apply {p:.3f} ms = "
          f"{nbytes / p / 8e9 * 100:.1f} % of 8 TB/s; max rel diff vs {a.libs[0]}: detect {dx:.2e}, apply {dy:.2e}",
          flush=True)
