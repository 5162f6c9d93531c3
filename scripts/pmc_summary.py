"""Summarise a scripts/gpu_profile.sh run into profiles/.

usage: python scripts/pmc_summary.py gpurun_out/prof_<tag> <tag> [notraffic]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.csv            per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch
  profiles/<tag>_summary.md         the two tables above plus the derived HBM traffic
  profiles/pmc_traffic.json         MRC-kernel HBM bytes per launch, read by bench.py
                                    (roofline.traffic) when its config matches

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  The factor
2 is the gfx950 correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE =
TCC_EA0_RDREQ x 64 B while the streaming reads are issued as 128-B requests.
It is calibrated for this kernel's 8-B/lane row loads: TCC_EA0_RDREQ x 128 B
matched the algorithmic IQ bytes within 2 % (profiles/README.md).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MRC = "k_mrc_td"
LS = "k_ls_td"


def short(name):
    n = name.split("(")[0].replace("void ", "")
    base, sep, targs = n.partition("<")
    return base.split("::")[-1] + sep + targs


def pmc(path, counter):
    acc = defaultdict(list)
    with open(path) as fp:
        for row in csv.DictReader(fp):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats_src = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    with open(stats_src) as fp:
        stats = list(csv.DictReader(fp))
    fetch, nf = pmc(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write, nw = pmc(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    with open(os.path.join(src, "bench_trace.json")) as fp:
        bench = json.loads([ln for ln in fp if ln.startswith("{")][-1])
    cfg = bench["config"]
    global MRC, LS
    if cfg.get("domain") == "freq":  # bench.py --mode freq
        MRC, LS = "k_mrc_freq", "k_ls_freq"
    one = cfg.get("flow") == "one-launch"  # bench.py's one-launch flow: k_demod_td<C> is the kernel
    if one:
        MRC = "k_demod_td"

    rows = []
    for k in sorted(fetch, key=lambda k: -fetch[k]):
        f_b = fetch[k] * 1024 * 2
        w_b = write.get(k, 0.0) * 1024
        rows.append((short(k), nf[k], fetch[k], write.get(k, 0.0), f_b + w_b))
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as fp:
        wr = csv.writer(fp)
        wr.writerow(["kernel", "dispatches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg",
                     "hbm_bytes_per_dispatch_corrected"])
        wr.writerows(rows)

    mrc = [r for r in rows if r[0].startswith(MRC)]
    mrc_stat = [s for s in stats if MRC in s["Name"]]
    ls_stat = [s for s in stats if LS in s["Name"]]
    q = cfg["data_symbols_per_gpu"]
    b_sym = cfg["R"] * cfg["C"] * 8 + (cfg["C"] - 1) * 8
    alg = q * b_sym
    if one:  # + the pilot symbol and pilot vector per frame
        alg += cfg["frames_per_gpu"] * (cfg["R"] * cfg["C"] * 8 + (cfg["C"] - 1) * 8)
    out = {"tag": tag, "config": dict({k: cfg[k] for k in ("R", "C", "S", "prefix", "frames_per_gpu")},
                                      domain=cfg.get("domain", "time"), flow=cfg.get("flow", "two-launch")),
           "mrc_kernel": mrc[0][0] if mrc else None,
           "mrc_hbm_bytes_per_launch": mrc[0][4] if mrc else None,
           "mrc_algorithmic_bytes_per_launch": alg,
           "mrc_avg_ns_rocprof": float(mrc_stat[0]["AverageNs"]) if mrc_stat else None,
           "ls_avg_ns_rocprof": float(ls_stat[0]["AverageNs"]) if ls_stat else None,
           "correction": "2*FETCH_SIZE + WRITE_SIZE (KiB->B); MI355X_MICROARCH.md HBM section",
           "build_id": bench.get("build_id"),  # the library the profiled run loaded (ofdm_lsmrc.build_id)
           "source": f"profiles/{tag}_pmc.csv"}
    if "notraffic" not in sys.argv[3:]:  # the default-config summary bench.py reads
        with open(os.path.join(prof, "pmc_traffic.json"), "w") as fp:
            json.dump(out, fp, indent=1)
    with open(os.path.join(prof, f"{tag}_traffic.json"), "w") as fp:
        json.dump(out, fp, indent=1)

    md = [f"# Profile {tag}", "",
          f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 1 --no-cpu` "
          f"(then one `--pmc FETCH_SIZE` and one `--pmc WRITE_SIZE` pass, `--steps 2`), "
          f"config {json.dumps(out['config'])}.", "",
          "## Kernel time (rocprofv3 --stats)", "",
          "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for s in stats:
        md.append(f"| {short(s['Name'])} | {s['Calls']} | {float(s['AverageNs']) / 1e6:.3f} | "
                  f"{float(s['Percentage']):.1f} |")
    md += ["", "## HBM traffic per dispatch (PMC, corrected)", "",
           "| kernel | dispatches | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM GB (2F+W) |", "|---|---|---|---|---|"]
    for r in rows:
        md.append(f"| {r[0]} | {r[1]} | {r[2]:.0f} | {r[3]:.0f} | {r[4] / 1e9:.3f} |")
    if mrc and mrc_stat:
        ns = float(mrc_stat[0]["AverageNs"])
        md += ["", f"MRC: algorithmic {alg / 1e9:.3f} GB/launch, measured HBM {mrc[0][4] / 1e9:.3f} GB/launch "
                   f"(ratio {mrc[0][4] / alg:.3f}); rocprof avg {ns / 1e6:.3f} ms -> "
                   f"{alg / ns:.0f} GB/s algorithmic ({alg / ns / 8000:.1%} of 8 TB/s), "
                   f"{mrc[0][4] / ns:.0f} GB/s measured."]
    md += ["", "bench line of the trace run:", "", "```", json.dumps(bench), "```", ""]
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as fp:
        fp.write("\n".join(md))
    print("\n".join(md))


if __name__ == "__main__":
    main()
