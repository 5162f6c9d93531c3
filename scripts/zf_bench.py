#!/usr/bin/env python3
"""Zero-forcing throughput on one MI355X.

Workload: U users x R antennas (default 16 x 64) over K = 1023 subcarriers.
  * precoder (createZeroForcingMatrix, cpuLS.hpp:415-447): one channel set
    per call, timed per call;
  * apply (multiplyWithChannelInv, cpuLS.hpp:449-463) and detect (its uplink
    counterpart) over `--nsym` symbols resident in HBM.
Roofline of apply / detect: HBM, algorithmic bytes per symbol = (U + R) * K *
8 (read the input symbol once, write the output once; W is an intermediate
re-read from L2) against 8 TB/s; their arithmetic, 8 * U * R * K flop per
symbol, is also reported against the 157.3 TFLOP/s f32 vector peak.  CPU
baseline: the oracle (the reference's cgemm/cgetrf/cgetri/cgemv sequence in
plain C, 1 thread) on a bounded sample."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"), os.path.join(ROOT, "tests")]

HBM_PEAK = 8.0e12
VALU_PEAK = 157.3e12


def timed(fn, reps):
    import torch
    fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--U", type=int, nargs="+", default=[16, 4, 8, 32])
    ap.add_argument("--R", type=int, default=64)
    ap.add_argument("--K", type=int, default=1023)
    ap.add_argument("--nsym", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ab", action="store_true",
                    help="round 3's A/B build only (OFDM_LSMRC_LIB=ab after scripts/experiments/ab_knobs_r3.patch)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import ofdm_lsmrc as ofdm
    from zf_cases import channel
    dev = torch.device("cuda:0")
    R, K, n = a.R, a.K, a.nsym
    res = {"config": {"workload": "zf", "R": R, "K": K, "nsym": n}, "by_users": {}}
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    Y = torch.randn((n, R, K), dtype=torch.complex64, device=dev, generator=g)
    for U in a.U:
        H = torch.from_numpy(channel(U, R, K, seed=U)).to(dev)
        W, Wt = ofdm.zf_precoder(H)
        X = torch.randn((n, U, K), dtype=torch.complex64, device=dev, generator=g)
        Xo = torch.empty_like(X)
        Yo = torch.empty_like(Y)
        t_pre = timed(lambda: ofdm.zf_precoder(H, W=W, Wt=Wt), a.reps)
        t_tr = timed(lambda: ofdm.zf_transpose(W), a.reps)
        ab = {}
        if a.ab:  # same-process A/B of the kernel variants (env knobs are read per launch)
            variants = {"lds": {"OFDM_AB_ZF_LDS": "1"}, "lds_8x4": {"OFDM_AB_ZF_LDS": "1", "OFDM_AB_ZF_ST": "4"},
                        "lds_nt": {"OFDM_AB_ZF_LDS": "1", "OFDM_AB_ZF_NT": "1"},
                        "dma": {"OFDM_AB_ZF_LDS": "2"}, "regtile": {"OFDM_AB_ZF_LDS": "0"},
                        "mfma_sg2": {"OFDM_AB_ZF_LDS": "3", "OFDM_AB_ZF_SG": "2"},
                        "mfma_sg4": {"OFDM_AB_ZF_LDS": "3", "OFDM_AB_ZF_SG": "4"},
                        "mfma_sg8": {"OFDM_AB_ZF_LDS": "3", "OFDM_AB_ZF_SG": "8"},
                        "mfma_lds_sg4": {"OFDM_AB_ZF_LDS": "4", "OFDM_AB_ZF_SG": "4"},
                        "mfma_lds_sg8": {"OFDM_AB_ZF_LDS": "4", "OFDM_AB_ZF_SG": "8"},
                        "mfma_lds8": {"OFDM_AB_ZF_LDS": "5"}, "mfma_lds8_m32": {"OFDM_AB_ZF_LDS": "6"}, "mfma_w128": {"OFDM_AB_ZF_LDS": "7"}, "mfma_wstat": {"OFDM_AB_ZF_LDS": "8"}, "mfma_wstat_xmap": {"OFDM_AB_ZF_LDS": "9"}, "mfma_wstat64": {"OFDM_AB_ZF_LDS": "10"}, "lds_xmap": {"OFDM_AB_ZF_LDS": "1", "OFDM_AB_ZF_XMAP": "1"},
                        }
            ref_d = ofdm.zf_detect(Wt, Y)  # default dispatch: every variant's outputs are checked against it
            ref_a = ofdm.zf_apply(Wt, X)
            diffs = {}
            for rnd in range(2):
                for key, env in variants.items():
                    for v in ("OFDM_AB_ZF_LDS", "OFDM_AB_ZF_NT", "OFDM_AB_ZF_ST", "OFDM_AB_ZF_SG", "OFDM_AB_ZF_XMAP"):
                        os.environ.pop(v, None)
                    os.environ.update(env)
                    d = timed(lambda: ofdm.zf_detect(Wt, Y, out=Xo), a.reps)
                    p = timed(lambda: ofdm.zf_apply(Wt, X, out=Yo), a.reps)
                    old = ab.get(key, (1e9, 1e9))
                    ab[key] = (min(old[0], d), min(old[1], p))
                    if rnd == 0:  # max |out - default| / max |default|, detect and apply
                        diffs[key] = [float((Xo - ref_d).abs().max() / ref_d.abs().max()),
                                      float((Yo - ref_a).abs().max() / ref_a.abs().max())]
            for v in ("OFDM_AB_ZF_LDS", "OFDM_AB_ZF_NT", "OFDM_AB_ZF_ST", "OFDM_AB_ZF_SG", "OFDM_AB_ZF_XMAP"):
                os.environ.pop(v, None)
        t_det = timed(lambda: ofdm.zf_detect(Wt, Y, out=Xo), a.reps)
        t_app = timed(lambda: ofdm.zf_apply(Wt, X, out=Yo), a.reps)
        byt = n * (U + R) * K * 8.0
        fl = 8.0 * U * R * K * n
        row = {"precoder_ms": t_pre, "transpose_ms": t_tr}
        if ab:
            row["ab_detect_apply_ms"] = ab
            row["ab_max_rel_diff_vs_default"] = diffs
        for name, t in (("detect", t_det), ("apply", t_app)):
            row[name] = {"ms": t, "symbols_per_s": n / (t * 1e-3),
                         "GBps": byt / (t * 1e-3) / 1e9, "hbm_frac": byt / (t * 1e-3) / HBM_PEAK,
                         "TFLOPs": fl / (t * 1e-3) / 1e12, "valu_frac": fl / (t * 1e-3) / VALU_PEAK}
        res["by_users"][str(U)] = row
        del X, Xo, Yo
    if not a.no_cpu:
        from oracle_bindings import Oracle
        from zf_cases import qpsk
        o = Oracle()
        U = a.U[0]
        Hn = channel(U, R, K, seed=U)
        t0 = time.perf_counter()
        Wn = o.zf_precoder(Hn)
        tp = time.perf_counter() - t0
        ns = 200
        Yn = qpsk(ns, R, K, seed=3)
        t0 = time.perf_counter()
        o.zf_detect(Wn, Yn)
        td = time.perf_counter() - t0
        res["cpu_baseline"] = {"precoder_ms": tp * 1e3, "detect_symbols_per_s": ns / td, "cores": 1,
                               "kind": "port", "sample": f"U={U} R={R} K={K}: 1 precoder, {ns} symbols detected"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
