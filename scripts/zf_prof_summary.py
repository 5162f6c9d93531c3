#!/usr/bin/env python3
"""Summarise scripts/r5/gpu_r5z.sh (ZF at U = 16, R = 64, K = 1023, 10 000
symbols): per kernel (detect k_zf_wstat, apply k_zf_apply_ws16) the rocprof
median dispatch time, % of 8 TB/s for the algorithmic (U + R) K 8 B per
symbol, HBM bytes from the PMC passes (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B,
the gfx950 correction of MI355X_MICROARCH.md), the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / dispatch time) and SQ wave-state fractions.
usage: python scripts/zf_prof_summary.py gpurun_out/r5z profiles/r5/r5z_zf"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

U, R, K, NSYM = 16, 64, 1023, 10000
ALG = (U + R) * K * 8 * NSYM
KERNELS = {"detect": "k_zf_wstat", "apply": "k_zf_apply_ws16"}


def rows(path):
    with open(path) as fp:
        yield from csv.DictReader(fp)


def find(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    raise FileNotFoundError(f"{d}/*{suffix}")


def per_dispatch(path, kname):
    per, dur = defaultdict(lambda: defaultdict(float)), {}
    for r in rows(path):
        if kname not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur


def main():
    src, dst = sys.argv[1], sys.argv[2]
    trace = find(os.path.join(src, "trace"), "kernel_trace.csv")
    out, lines = {}, []
    for role, kname in KERNELS.items():
        ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows(trace) if kname in r["Kernel_Name"])
        med = ds[len(ds) // 2] * 1e-9
        f, _ = per_dispatch(find(os.path.join(src, "pmc_FETCH_SIZE"), "counter_collection.csv"), kname)
        w, _ = per_dispatch(find(os.path.join(src, "pmc_WRITE_SIZE"), "counter_collection.csv"), kname)
        g, gd = per_dispatch(find(os.path.join(src, "pmc_GRBM_GUI_ACTIVE"), "counter_collection.csv"), kname)
        fetch = statistics.median(v["FETCH_SIZE"] for v in f.values()) * 1024
        write = statistics.median(v["WRITE_SIZE"] for v in w.values()) * 1024
        hbm = 2 * fetch + write
        ghz = statistics.median(v["GRBM_GUI_ACTIVE"] / 8 / gd[i] for i, v in g.items())
        sq = {c: statistics.median(v[c] / v["SQ_WAVE_CYCLES"] for v in g.values())
              for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")}
        out[role] = {"kernel": kname, "dispatches": len(ds), "median_ms": med * 1e3,
                     "achieved_GBps": ALG / med / 1e9, "frac_of_8TBps": ALG / med / 8e12,
                     "hbm_bytes_pmc": hbm, "traffic_over_algorithmic": hbm / ALG, "effective_GHz": ghz, **sq}
        lines.append(f"| {role} (`{kname}`) | {len(ds)} | {med*1e3:.3f} | {ALG/med/1e9:.0f} GB/s = {100*ALG/med/8e12:.1f} % | "
                     f"{hbm/1e9:.3f} GB = {hbm/ALG:.3f}x | {ghz:.2f} GHz | {sq['SQ_WAIT_ANY']:.2f} / {sq['SQ_ACTIVE_INST_VALU']:.2f} / {sq['SQ_ACTIVE_INST_LDS']:.2f} |")
    bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    with open(dst + "_summary.md", "w") as fp:
        fp.write(f"# ZF profile ({os.path.basename(src)})\n\nU = {U}, R = {R}, K = {K}, {NSYM} symbols; algorithmic bytes "
                 f"(U + R) K 8 per symbol = {ALG/1e9:.3f} GB per call.  `scripts/r5/gpu_r5z.sh`, `scripts/zf_prof_summary.py`.\n\n"
                 "| op | dispatches | rocprof median ms | achieved | HBM (PMC, 2F+W) | clock | WAIT_ANY / VALU / LDS |\n|---|---|---|---|---|---|---|\n")
        fp.write("\n".join(lines) + "\n\nbench line (un-profiled run):\n\n```\n" + bench + "\n```\n")
    with open(dst + "_pmc.json", "w") as fp:
        json.dump(out, fp, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
