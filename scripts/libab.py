#!/usr/bin/env python3
"""Compare builds of the same sources with different compiler options
(lib/libofdm_lsmrc_<name>.so, made with `make EXTRA=... OBJDIR=... LIB=...`):
scripts/ab.py's default kernels, one process per (shape, build), builds
interleaved over repetitions on the same box.

usage: python scripts/libab.py [--reps 2] NAME [NAME ...]   ("" = the product build)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--shapes", default="1024:64:400,2048:64:400,4096:32:300", help="C:R:frames,...")
ap.add_argument("--extra", default="", help="more scripts/ab.py arguments, e.g. --ls")
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
libs = ["" if x in ("prod", '""') else x for x in a.libs]
res = {}
for shape in a.shapes.split(","):
    C, R, F = shape.split(":")
    for rep in range(a.reps):
        for lib in libs:
            env = dict(os.environ, OFDM_LSMRC_LIB=lib)
            p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "scripts", "ab.py"), "--C", C, "--R", R,
                                "--frames", F, "--reps", "3"] + a.extra.split() + ["default"], env=env, capture_output=True, text=True,
                               timeout=240)
            if p.returncode != 0:
                print(p.stdout, p.stderr, flush=True)
                sys.exit(p.returncode)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
            d = json.loads(line)
            d["lib"] = lib or "prod"
            d["rep"] = rep
            print(json.dumps(d), flush=True)
            res.setdefault((C, lib or "prod"), []).append(d["ms"])
for (C, lib), v in res.items():
    print(f"C={C} {lib}: {' '.join(f'{x:.3f}' for x in v)} ms", flush=True)
