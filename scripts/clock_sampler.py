#!/usr/bin/env python3
"""Sample the GPU shader clock while a command runs (evidence for the clock a
bench or profile ran at): `python scripts/clock_sampler.py OUT.jsonl -- cmd ...`
starts `cmd` as a child, polls `rocm-smi --showclocks --json` every --period
seconds until it exits, writes one JSON line per sample, prints a summary
(median / min / max sclk MHz over the samples) and exits with the child's
status.  The sampler itself never touches the GPU through HIP."""
import json
import statistics
import subprocess
import sys
import time


def sclk():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=10)
        d = json.loads(r.stdout)
    except Exception:
        return None
    out = {}
    for card, v in d.items():
        for k, s in v.items():
            if "sclk" in k.lower() and "(" in str(s):
                try:
                    out[card] = float(str(s).split("(")[1].split("Mhz")[0].split("MHz")[0])
                except ValueError:
                    pass
    return out


def main():
    out_path = sys.argv[1]
    period = 0.25
    cmd = sys.argv[sys.argv.index("--") + 1:]
    p = subprocess.Popen(cmd)
    samples = []
    with open(out_path, "w") as fp:
        while p.poll() is None:
            s = sclk()
            if s:
                rec = {"t": time.time(), "sclk_mhz": s}
                samples.append(rec)
                fp.write(json.dumps(rec) + "\n")
                fp.flush()
            time.sleep(period)
    vals = [v for r in samples for v in r["sclk_mhz"].values()]
    busy = [v for v in vals if v > 500]
    if vals:
        print(json.dumps({"clock_samples": len(vals), "sclk_mhz_median": statistics.median(vals),
                          "sclk_mhz_median_busy": statistics.median(busy) if busy else None,
                          "sclk_mhz_max": max(vals), "sclk_mhz_min": min(vals)}), file=sys.stderr)
    sys.exit(p.returncode)


if __name__ == "__main__":
    main()
