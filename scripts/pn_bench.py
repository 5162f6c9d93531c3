#!/usr/bin/env python3
"""PN frame-sync correlator throughput on one MI355X.

Workload: rx_and_corr.cpp's search over R channels of an N-sample receive
buffer for an L-tap PN (defaults: R=64, N=110,000 -- one 101-symbol frame of
1024+72 samples plus the PN --, L=1023), no hit, so every lag of every channel
is evaluated (the worst case; a hit in channel 0 stops the reference early and
this kernel's later workgroups exit too).  Reported: lags/s, and the VALU
roofline: 8 non-fused f32 ops per complex tap (the reference's exact
arithmetic, no FMA) against 78.6 T ops/s (1024 SIMDs x 32 lanes x 2.4 GHz;
the 157.3 TFLOPS vector peak counts an FMA as 2).  CPU baseline: the oracle
(the reference's loop, single thread as in rx_and_corr) on channel 0's first
`--cpu-lags` lags."""
import argparse
import json
import os
os.environ.setdefault("OFDM_LSMRC_LIB", "ab")  # the A/B build: OFDM_AB_* switches
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"), os.path.join(ROOT, "tests")]

VALU_PEAK_OPS = 1024 * 32 * 2.4e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=64)
    ap.add_argument("--N", type=int, default=110000)
    ap.add_argument("--L", type=int, default=1023)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-lags", type=int, default=4000)
    a = ap.parse_args()
    import numpy as np
    import torch
    import ofdm_lsmrc as ofdm
    from pn_cases import rx_buffer
    dev = torch.device("cuda:0")
    buf, pn = rx_buffer(a.R, a.N, a.L, {}, noise=0.05)
    db, dp = torch.from_numpy(buf).to(dev), torch.from_numpy(pn).to(dev)
    nl = a.N - a.L + 1
    res = {}
    # A/B of the exact MAC form (packed VOP3P vs scalar; bit-identical), same process
    ab = {}
    for pk in ("0", "1", "0", "1"):
        os.environ["OFDM_AB_PN_PK"] = pk
        ofdm.pn_correlate(db, dp, 0.5)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ofdm.pn_correlate(db, dp, 0.5)
        e1.record()
        torch.cuda.synchronize()
        ab["packed" if pk == "1" else "scalar"] = e0.elapsed_time(e1) / a.reps
    os.environ.pop("OFDM_AB_PN_PK")
    res["ab_ms"] = ab
    for want_mag in (False, True):
        pos, _ = ofdm.pn_correlate(db, dp, 0.5, mag=want_mag)  # warm-up
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            pos, _ = ofdm.pn_correlate(db, dp, 0.5, mag=want_mag)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        ops = a.R * nl * a.L * 8.0
        res["store_mag" if want_mag else "search"] = {
            "ms": ms, "lags_per_s": a.R * nl / (ms * 1e-3),
            "valu_Tops": ops / (ms * 1e-3) / 1e12, "valu_frac": ops / (ms * 1e-3) / VALU_PEAK_OPS,
            "pos": int(pos.item())}
    from oracle_bindings import Oracle
    o = Oracle()
    sub = buf[:1, :a.cpu_lags + a.L - 1]
    t0 = time.perf_counter()
    o.pn_correlate(sub, pn, 1e30)
    cs = time.perf_counter() - t0
    res["cpu_baseline"] = {"lags_per_s": a.cpu_lags / cs, "cores": 1, "kind": "port",
                           "sample": f"{a.cpu_lags} lags of one channel, L={a.L}"}
    res["config"] = {"R": a.R, "N": a.N, "L": a.L, "lags": a.R * nl}
    res["speedup_vs_cpu"] = res["search"]["lags_per_s"] / res["cpu_baseline"]["lags_per_s"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
