#!/usr/bin/env python3
"""ZF detect / apply with row pitches (ofdm_zf_detect_ex / _apply_ex) against the reference layout,
same process, alternating: U users x R antennas x K subcarriers, nsym symbols
in HBM.  Algorithmic bytes (U + R) K 8 per symbol in every layout (the pad is
neither read nor written).  usage: python scripts/zf_pitch_ab.py [--U 16] [--reps 5]"""
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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--launches", type=int, default=10)
ap.add_argument("--op", choices=["detect", "apply"], default="detect")
a = ap.parse_args()

import torch  # noqa: E402
import ofdm_lsmrc as ofdm  # noqa: E402
from zf_cases import channel  # noqa: E402

dev = torch.device("cuda:0")
U, R, K, n = a.U, a.R, a.K, a.nsym
_, Wt = ofdm.zf_precoder(torch.from_numpy(channel(U, R, K, seed=U)).to(dev), W=False)
g = torch.Generator(device=dev)
g.manual_seed(0)
Kp = (K + 15) // 16 * 16
if a.op == "detect":
    Ypad = torch.randn((n, R, Kp), dtype=torch.complex64, device=dev, generator=g)
    Y = Ypad[:, :, :K].contiguous()
    ref = ofdm.zf_detect(Wt, Y)
    cases = {
        "reference layout (ldy = ldx = K)": (lambda o: ofdm.zf_detect(Wt, Y, out=o), (n, U, K), Y),
        f"ldy = K, ldx = {Kp}": (lambda o: ofdm.zf_detect_pitched(Wt, Y, out=o), (n, U, Kp), Y),
        f"ldy = ldx = {Kp}": (lambda o: ofdm.zf_detect_pitched(Wt, Ypad, out=o), (n, U, Kp), Ypad),
    }
else:
    Xpad = torch.randn((n, U, Kp), dtype=torch.complex64, device=dev, generator=g)
    X = Xpad[:, :, :K].contiguous()
    ref = ofdm.zf_apply(Wt, X)
    cases = {
        "reference layout (ldx = ldy = K)": (lambda o: ofdm.zf_apply(Wt, X, out=o), (n, R, K), X),
        f"ldx = K, ldy = {Kp}": (lambda o: ofdm.zf_apply_pitched(Wt, X, out=o), (n, R, Kp), X),
        f"ldx = ldy = {Kp}": (lambda o: ofdm.zf_apply_pitched(Wt, Xpad, out=o), (n, R, Kp), Xpad),
    }
outs = {k: torch.empty(shape, dtype=torch.complex64, device=dev) for k, (_, shape, _) in cases.items()}
byt = n * (U + R) * K * 8.0
res = {k: [] for k in cases}
s = torch.cuda.current_stream()
for rep in range(a.reps):
    for name, (fn, _, _) in (list(cases.items()) if rep % 2 == 0 else list(cases.items())[::-1]):
        fn(outs[name])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.launches):
            fn(outs[name])
        e1.record(s)
        torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / a.launches)
for name, v in res.items():
    m = sorted(v)[len(v) // 2]
    same = bool(torch.equal(outs[name][:, :, :K], ref))
    print(json.dumps({"op": a.op, "layout": name, "U": U, "R": R, "K": K, "nsym": n, "ms_median": m, "ms_all": v,
                      "TBps": byt / m / 1e9, "hbm_frac": byt / m / 8e9, "bit_identical_to_reference_layout": same}),
          flush=True)
