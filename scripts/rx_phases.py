#!/usr/bin/env python3
"""Phases of the one-launch demod's receiver workgroups from the diagnostic
build's stamps (bench.py --stamps-out X.npy; frame_td.hip k_demod_td1024:
MARKN(0) ticket taken, MARKN(1) tables filled and row 0's DMA issued, MARK
estimate seen, MARKN(2) rows done (whole blocks only; half units return
before it), end after the epilogue).  usage: python scripts/rx_phases.py X.npy NLS

Prints, for whole blocks of the first round (started < 5 us) and of the
later rounds, p10 / p50 / p90 of each phase in us, and the share of a
later block's lifetime spent before its first row."""
import sys

import numpy as np

rec = np.load(sys.argv[1]).astype(np.int64)
nls = int(sys.argv[2])
rec = rec[rec[:, 2] > 0]
t0 = rec[:, 0].min()
blk = rec[:, 7] & 0xFFFFFFFF
rx = rec[(blk >= nls) & (rec[:, 10] > 0) & (rec[:, 8] > 0) & (rec[:, 9] > 0)]
us = lambda a: a * 1e-2
start = us(rx[:, 0] - t0)
phases = {
    "ticket": us(rx[:, 8] - rx[:, 0]),
    "fill+dma": us(rx[:, 9] - rx[:, 8]),
    "flag": us(rx[:, 1] - rx[:, 9]),
    "rows": us(rx[:, 10] - rx[:, 1]),
    "epilogue": us(rx[:, 2] - rx[:, 10]),
    "life": us(rx[:, 2] - rx[:, 0]),
}
for name, m in (("first round", start < 5.0), ("later", start >= 5.0)):
    print(f"{name}: {int(m.sum())} whole blocks")
    for k, v in phases.items():
        p = np.percentile(v[m], [10, 50, 90]) if m.any() else [0, 0, 0]
        print(f"  {k:9s} p10 {p[0]:7.2f}  p50 {p[1]:7.2f}  p90 {p[2]:7.2f} us")
m = start >= 5.0
if m.any():
    pre = phases["ticket"] + phases["fill+dma"] + phases["flag"]
    print(f"later blocks: start-to-first-row {np.median(pre[m]):.2f} us of {np.median(phases['life'][m]):.2f} us "
          f"({100 * np.median(pre[m] / phases['life'][m]):.1f} %)")
