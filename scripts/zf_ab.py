#!/usr/bin/env python3
"""Same-process A/B of ZF apply/detect variants of the A/B build:
python scripts/zf_ab.py [--U 16] [--nsym 10000] default NAME=VAL[,NAME=VAL] ...
One JSON line per variant: detect / apply ms (best of 3 x `--reps`) and the max
relative difference from the first variant."""
import argparse
import json
import os
import sys

os.environ["OFDM_LSMRC_LIB"] = "ab"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"), os.path.join(ROOT, "tests")]
ap = argparse.ArgumentParser()
ap.add_argument("--U", type=int, default=16)
ap.add_argument("--R", type=int, default=64)
ap.add_argument("--K", type=int, default=1023)
ap.add_argument("--nsym", type=int, default=10000)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("variants", nargs="*", default=["default"])
a = ap.parse_args()
import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402
from zf_cases import channel  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(0)
U, R, K, n = a.U, a.R, a.K, a.nsym
Y = torch.randn((n, R, K), dtype=torch.complex64, device=dev, generator=g)
X = torch.randn((n, U, K), dtype=torch.complex64, device=dev, generator=g)
W, Wt = ofdm.zf_precoder(torch.from_numpy(channel(U, R, K, seed=U)).to(dev))
Xo, Yo = torch.empty_like(X), torch.empty_like(Y)
keys = {kv.split("=")[0] for v in a.variants if v != "default" for kv in v.split(",")}


def timed(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps


best, diff, ref = {}, {}, None
for rnd in range(3):
    for v in a.variants:
        for k in keys:
            os.environ.pop("OFDM_AB_" + k, None)
        if v != "default":
            for kv in v.split(","):
                k, val = kv.split("=")
                os.environ["OFDM_AB_" + k] = val
        d = timed(lambda: ofdm.zf_detect(Wt, Y, out=Xo))
        p = timed(lambda: ofdm.zf_apply(Wt, X, out=Yo))
        o = best.get(v, (1e9, 1e9))
        best[v] = (min(o[0], d), min(o[1], p))
        if rnd == 0:
            if ref is None:
                ref = (Xo.clone(), Yo.clone())
            diff[v] = [float((Xo - ref[0]).abs().max() / ref[0].abs().max()),
                       float((Yo - ref[1]).abs().max() / ref[1].abs().max())]
byt = n * (U + R) * K * 8.0
for v in a.variants:
    d, p = best[v]
    print(json.dumps({"variant": v, "U": U, "R": R, "nsym": n, "detect_ms": round(d, 4), "apply_ms": round(p, 4),
                      "detect_frac": round(byt / (d * 1e-3) / 8e12, 4), "apply_frac": round(byt / (p * 1e-3) / 8e12, 4),
                      "max_rel_diff_vs_first": diff[v]}), flush=True)
