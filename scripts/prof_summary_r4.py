#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof_r4.sh run into profiles/r4/.

usage: python scripts/prof_summary_r4.py gpurun_out/prof_<tag> <tag> [traffic]

Writes profiles/r4/<tag>_summary.md, <tag>_kernel_stats.csv (rocprofv3
--stats, copied), <tag>_dispatches.csv (per-dispatch durations of the
dominant kernel from the trace run) and <tag>_pmc.json; with `traffic` also
profiles/pmc_traffic.json (what bench.py reports as roofline.traffic for the
default configuration).

HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B): the gfx950
correction of MI355X_MICROARCH.md (FETCH_SIZE counts 64-B units of reads that
are issued as 128-B requests; calibrated for these kernels in profiles/README.md).
Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time
(MI355X_MICROARCH.md, DVFS give-back).
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0].replace("void ", "")
    base, sep, targs = n.partition("<")
    return base.split("::")[-1] + sep + targs


def last_json(path):
    with open(path) as fp:
        lines = [ln for ln in fp if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


BIG_ONLY = False  # split mode: only the whole-batch launches (>= half the longest) of the dominant kernel


def counters(path):
    """{kernel: {counter: [values per dispatch]}}, {kernel: [durations ns]}"""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    dur = defaultdict(dict)
    with open(path) as fp:
        for row in csv.DictReader(fp):
            k = short(row["Kernel_Name"])
            per[k][row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
            dur[k][row["Dispatch_Id"]] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    vals = defaultdict(lambda: defaultdict(list))
    durs = {}
    for k, d in dur.items():
        cut = 0.5 * max(d.values()) if BIG_ONLY else -1
        keep = [i for i in d if d[i] >= cut]
        for i in keep:
            for c, v in per[k][i].items():
                vals[k][c].append(v)
        durs[k] = [d[i] for i in keep]
    return vals, durs


def dominant(bench):
    cfg = bench["config"]
    if "R_total" in cfg:  # split mode: the partial-numerator MRC
        return {1024: "k_mrc_td1024_hlds", 2048: "k_mrc_td2048", 4096: "k_mrc_td4096h",
                1536: "k_mrc_td1536", 3072: "k_mrc_td3072", 6144: "k_mrc_td6144", 512: "k_mrc_td512", 256: "k_mrc_td256", 128: "k_mrc_td128"}.get(cfg["C"], "k_mrc_any")
    if cfg.get("domain") == "freq":
        return "k_mrc_freq"
    if cfg.get("flow") == "one-launch":
        return "k_demod_td"
    return {1024: "k_mrc_td1024_hlds", 2048: "k_mrc_td2048", 4096: "k_mrc_td4096h",
            1536: "k_mrc_td1536", 3072: "k_mrc_td3072", 6144: "k_mrc_td6144", 512: "k_mrc_td512", 256: "k_mrc_td256", 128: "k_mrc_td128"}.get(cfg["C"], "k_mrc_any")


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles", tag[:2] if tag[:1] == "r" and tag[1:2].isdigit() else "r4")
    os.makedirs(prof, exist_ok=True)
    args = open(os.path.join(src, "args.txt")).read().strip()
    unprof = last_json(os.path.join(src, "bench_unprofiled.json"))
    traced = last_json(os.path.join(src, "bench_trace.json"))
    kern = dominant(traced)
    cfg = traced["config"]
    global BIG_ONLY
    BIG_ONLY = "R_total" in cfg
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as fp:
        stats = list(csv.DictReader(fp))
    # per-dispatch durations of the dominant kernel in the trace run
    durs = []
    with open(os.path.join(src, "trace", "run_kernel_trace.csv")) as fp:
        for row in csv.DictReader(fp):
            if short(row["Kernel_Name"]).startswith(kern):
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if BIG_ONLY and durs:  # the pipeline's per-chunk launches are not the roofline kernel's
        durs = [d for d in durs if d >= 0.5 * max(durs)]
    with open(os.path.join(prof, f"{tag}_dispatches.csv"), "w", newline="") as fp:
        w = csv.writer(fp)
        w.writerow(["dispatch", "kernel", "ns"])
        for i, d in enumerate(durs):
            w.writerow([i, kern, d])
    # PMC passes
    fetch, fdur = counters(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write, _ = counters(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    sq, sqdur = counters(os.path.join(src, "pmc_GRBM_GUI_ACTIVE", "run_counter_collection.csv"))
    k_f = next(k for k in fetch if k.startswith(kern))
    fetch_kib = statistics.mean(fetch[k_f]["FETCH_SIZE"])
    write_kib = statistics.mean(write[k_f]["WRITE_SIZE"])
    hbm = fetch_kib * 1024 * 2 + write_kib * 1024
    k_s = next(k for k in sq if k.startswith(kern))
    s = {c: statistics.mean(v) for c, v in sq[k_s].items()}
    sq_ns = statistics.mean(sqdur[k_s])
    clock_ghz = s["GRBM_GUI_ACTIVE"] / 8 / sq_ns
    wave = s.get("SQ_WAVE_CYCLES", 0.0)
    frac = {c: s[c] / wave for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                      "SQ_ACTIVE_INST_LDS") if c in s and wave}
    b_sym = cfg.get("R", cfg.get("R_per_gpu")) * cfg["C"] * 8 + (cfg["C"] - 1) * 8
    q = cfg.get("data_symbols_per_gpu", cfg.get("data_symbols"))
    alg = q * b_sym
    if kern == "k_demod_td":
        alg += cfg["frames_per_gpu"] * b_sym
    avg_ns = statistics.mean(durs)
    med_ns = statistics.median(durs)
    # the timed steps only: the last `steps` dispatches of the trace run
    steps = traced["steps"]
    # split mode: the bench's 5 roofline launches over the whole local batch come last
    timed = durs[-5:] if "R_total" in cfg else durs[-steps:]
    out = {"tag": tag, "command": f"python3 bench.py {args}", "kernel": kern,
           "config": {k: cfg[k] for k in cfg if k != "workload"},
           "rocprof_avg_ms_all": avg_ns / 1e6, "rocprof_median_ms_all": med_ns / 1e6, "dispatches": len(durs),
           "rocprof_avg_ms_timed_steps": statistics.mean(timed) / 1e6,
           "rocprof_median_ms_timed_steps": statistics.median(timed) / 1e6,
           "bench_profiled_ms_per_step": traced["ms_per_step"],
           "bench_profiled_event_avg_ms": traced.get("roofline", {}).get("avg_launch_ms"),
           "bench_unprofiled_ms_per_step": unprof["ms_per_step"] if unprof else None,
           "bench_unprofiled_event_avg_ms": (unprof or {}).get("roofline", {}).get("avg_launch_ms"),
           "algorithmic_bytes_per_launch": alg,
           "hbm_bytes_per_launch": hbm, "hbm_over_algorithmic": hbm / alg,
           "mrc_hbm_bytes_per_launch": hbm, "mrc_algorithmic_bytes_per_launch": alg,
           "effective_clock_ghz_pmc_pass": clock_ghz, "sq_fractions_of_wave_cycles": frac,
           "correction": "2*FETCH_SIZE + WRITE_SIZE (KiB->B); MI355X_MICROARCH.md HBM section",
           "build_id": traced.get("build_id")}  # the library the profiled run loaded (ofdm_lsmrc.build_id)
    clk = os.path.join(src, "clock_unprofiled.jsonl")
    if os.path.exists(clk):
        vals = []
        with open(clk) as fp:
            for ln in fp:
                vals += list(json.loads(ln)["sclk_mhz"].values())
        busy = [v for v in vals if v > 500]
        out["rocm_smi_sclk_mhz_unprofiled"] = {"samples": len(vals), "median_busy": statistics.median(busy)
                                               if busy else None, "max": max(vals) if vals else None}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as fp:
        json.dump(out, fp, indent=1)
    if "frames_per_gpu" in cfg:  # frames / freq modes: a traffic record bench.py can attach (same build only)
        t = {"tag": tag, "config": {"R": cfg["R"], "C": cfg["C"], "S": cfg["S"], "prefix": cfg["prefix"],
                                    "frames_per_gpu": cfg["frames_per_gpu"], "domain": cfg.get("domain", "time"),
                                    "flow": cfg.get("flow", "two-launch")},
             "mrc_kernel": kern, "mrc_hbm_bytes_per_launch": hbm, "mrc_algorithmic_bytes_per_launch": alg,
             "mrc_avg_ns_rocprof": avg_ns, "correction": out["correction"], "build_id": out["build_id"],
             "source": os.path.relpath(os.path.join(prof, f"{tag}_pmc.json"), ROOT)}
        with open(os.path.join(prof, f"{tag}_traffic.json"), "w") as fp:
            json.dump(t, fp, indent=1)
        if "traffic" in sys.argv[3:]:  # the default shape's record
            with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fp:
                json.dump(t, fp, indent=1)
    md = [f"# Profile {tag}", "",
          f"Command (driver form): `python3 bench.py {args}`, run three ways in ONE GPU session: un-profiled, "
          f"under `rocprofv3 --kernel-trace --stats`, and under `rocprofv3 --kernel-trace --pmc ...` "
          f"(FETCH_SIZE; WRITE_SIZE; GRBM_GUI_ACTIVE + 8 SQ counters; `--no-cpu --no-mode-a` in the PMC passes).", "",
          f"Dominant kernel `{kern}`; algorithmic bytes per launch {alg / 1e9:.3f} GB.", "",
          "| quantity | value |", "|---|---|",
          f"| rocprof avg / median per dispatch (all {len(durs)}) | {avg_ns / 1e6:.3f} / {med_ns / 1e6:.3f} ms |",
          f"| rocprof avg / median, the {len(timed)} timed-step dispatches | "
          f"{out['rocprof_avg_ms_timed_steps']:.3f} / {out['rocprof_median_ms_timed_steps']:.3f} ms |",
          f"| bench ms_per_step in the profiled process | {traced['ms_per_step']:.3f} ms |",
          f"| bench ms_per_step un-profiled (same session, before) | "
          f"{unprof['ms_per_step'] if unprof else float('nan'):.3f} ms |",
          f"| achieved (algorithmic / rocprof median) | {alg / med_ns:.0f} GB/s = {alg / med_ns / 8000:.1%} of 8 TB/s |",
          f"| HBM bytes per launch (PMC, 2F+W) | {hbm / 1e9:.3f} GB = {hbm / alg:.3f} x algorithmic |",
          f"| effective clock in the PMC pass (GRBM_GUI_ACTIVE / 8 / wall) | {clock_ghz:.2f} GHz |"]
    if "rocm_smi_sclk_mhz_unprofiled" in out:
        r = out["rocm_smi_sclk_mhz_unprofiled"]
        md.append(f"| rocm-smi sclk during the un-profiled run (median of busy samples) | {r['median_busy']} MHz "
                  f"({r['samples']} samples) |")
    for c, v in frac.items():
        md.append(f"| {c} / SQ_WAVE_CYCLES | {v:.3f} |")
    md += ["", "## Kernel time (rocprofv3 --stats of the trace run)", "",
           "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for st in stats:
        md.append(f"| {short(st['Name'])} | {st['Calls']} | {float(st['AverageNs']) / 1e6:.3f} | "
                  f"{float(st['Percentage']):.1f} |")
    md += ["", "bench line of the profiled run:", "", "```", json.dumps(traced), "```", "",
           "bench line of the un-profiled run:", "", "```", json.dumps(unprof), "```", ""]
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as fp:
        fp.write("\n".join(md))
    print("\n".join(md[:20]))


if __name__ == "__main__":
    main()
