#!/usr/bin/env python3
"""rocprofv3 kernel trace of the reference's frame flow through the drop-in
headers: a ring writer process feeds one frame of the
golden fixture, tests/cpp/e2e_reader.cpp runs gpuLS::demodOneFrame (the
reference's demodOneFrameCUDA path) under
`rocprofv3 --kernel-trace --stats`, and its Output_gpu.dat is checked against
the golden output.  The kernel list must be the fused LS + MRC pair only.
usage: python scripts/frame_flow_trace.py <out dir> [fixture] [flow]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import GOLDEN, parity  # noqa: E402
from test_e2e_gpu import build, raw_pilots  # noqa: E402

out = os.path.abspath(sys.argv[1])
fixture = sys.argv[2] if len(sys.argv) > 2 else "cfg1_r4_c1024_s10"
flow = sys.argv[3] if len(sys.argv) > 3 else "frame"
os.makedirs(out, exist_ok=True)
z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
iq = z["iq"][0]
S, R, Cp = iq.shape
prefix = int(z["prefix"])
C = Cp - prefix
raw_pilots(z["X"]).astype(np.complex64).tofile(os.path.join(out, "Pilots.dat"))
iq.astype(np.complex64).tofile(os.path.join(out, "iq.bin"))
shm = f"/ofdm_trace_{os.getpid()}"
writer = build(out, "e2e_writer", R, C, prefix, S, shm)
reader = build(out, "e2e_reader", R, C, prefix, S, shm)
w = subprocess.Popen([writer, "iq.bin"], cwd=out, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
try:
    r = subprocess.run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d",
                        os.path.join(out, "trace"), "-o", "run", "--", reader, flow],
                       cwd=out, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    w.communicate(timeout=60)
finally:
    if w.poll() is None:
        w.kill()
got = np.fromfile(os.path.join(out, "Output_gpu.dat"), np.complex64).reshape(S - 1, C - 1)
parity(got, z["out"][0])
print("Output_gpu.dat matches the golden output")
import csv  # noqa: E402
import glob  # noqa: E402
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        print(row["Name"].split("(")[0], row["Calls"], row["AverageNs"])
