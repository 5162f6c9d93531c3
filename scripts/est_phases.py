#!/usr/bin/env python3
"""Phases of the one-launch demod's estimator workgroups from the diagnostic
build's stamps (bench.py --stamps-out X.npy): start -> tables filled (mark
n0) -> first pilot row done (p1) -> all rows (p2) -> |H|^2 stored (p3) ->
flag published (mark) -> end; and of the first round's receivers: start ->
estimate seen (mark) -> end.  usage: python scripts/est_phases.py X.npy NLS"""
import sys

import numpy as np

rec = np.load(sys.argv[1]).astype(np.int64)
nls = int(sys.argv[2])
rec = rec[rec[:, 2] > 0]
t0 = rec[:, 0].min()
us = lambda c: (c - t0) * 1e-2
blk = rec[:, 7] & 0xFFFFFFFF
est = rec[blk < nls]
cols = {"start": 0, "fill": 8, "row1": 9, "rows": 10, "P": 11, "publish": 1, "end": 2}
prev = None
print(f"estimators: {len(est)}")
for name, c in cols.items():
    v = us(est[:, c])
    v = v[est[:, c] > 0]
    p = np.percentile(v, [10, 50, 90])
    print(f"  {name:8s} at p10 {p[0]:7.2f}  p50 {p[1]:7.2f}  p90 {p[2]:7.2f} us")
mrc = rec[blk >= nls]
first = mrc[us(mrc[:, 0]) < 5.0]
print(f"first-round receivers (started < 5 us): {len(first)}")
for name, c in (("start", 0), ("estimate seen", 1), ("end", 2)):
    p = np.percentile(us(first[:, c]), [10, 50, 90])
    print(f"  {name:14s} at p10 {p[0]:7.2f}  p50 {p[1]:7.2f}  p90 {p[2]:7.2f} us")
