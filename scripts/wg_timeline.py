#!/usr/bin/env python3
"""Workgroup timeline of one launch from the diagnostic build's stamps
(bench.py --stamps-out X.npy; csrc/diag.hpp: per workgroup rt_start, rt_mark,
rt_end in 100 MHz ticks, mt_start / mt_end shader clock, hw_id, xcc_id,
block).

usage: python scripts/wg_timeline.py X.npy [--nls N] [--json]
  --nls N   the first N blocks are the one-launch kernel's estimator
            workgroups (k_demod_td1024: nframes rounded up to 8)
Prints: span, per-role start / wait / work / end statistics (us), the
active-workgroup curve in 10 equal time slices, the time the last
workgroups run alone (tail: from when the active count falls below half its
peak), and the effective clock per role.
"""
import argparse
import json

import numpy as np


def analyse(rec, nls=0):
    rec = rec[rec[:, 2] > 0].astype(np.int64)
    t0 = rec[:, 0].min()
    st = (rec[:, 0] - t0) * 1e-2  # us
    mk = (rec[:, 1] - t0) * 1e-2
    en = (rec[:, 2] - t0) * 1e-2
    ghz = (rec[:, 4] - rec[:, 3]) / np.maximum(rec[:, 2] - rec[:, 0], 1) * 0.1
    blk = rec[:, 7] & 0xFFFFFFFF
    span = en.max()
    res = {"workgroups": int(len(rec)), "span_us": float(span)}
    roles = {"all": np.ones(len(rec), bool)}
    if nls:
        roles = {"estimator": blk < nls, "mrc": blk >= nls}
    for name, m in roles.items():
        if not m.any():
            continue
        q = lambda a: [float(np.percentile(a[m], p)) for p in (0, 10, 50, 90, 100)]
        res[name] = {"n": int(m.sum()), "start_us_p0_10_50_90_100": q(st), "end_us": q(en),
                     "mark_minus_start_us": q(mk - st), "end_minus_mark_us": q(en - mk),
                     "life_us": q(en - st), "GHz_median": float(np.median(ghz[m]))}
    # active workgroups over time
    ts = np.linspace(0, span, 201)
    act = np.array([((st <= t) & (en > t)).sum() for t in ts])
    peak = act.max()
    res["active_peak"] = int(peak)
    res["active_by_tenth"] = [int(act[i * 20:(i + 1) * 20].mean()) for i in range(10)]
    below = np.nonzero((act < peak / 2) & (ts > ts[np.argmax(act)]))[0]
    res["tail_us_below_half_peak"] = float(span - ts[below[0]]) if len(below) else 0.0
    # first-round start: when the active count first reaches 90 % of its peak
    up = np.nonzero(act >= 0.9 * peak)[0]
    res["ramp_us_to_90pct"] = float(ts[up[0]]) if len(up) else None
    # work-weighted occupancy: sum of lifetimes / (peak x span)
    res["occupancy_fill"] = float((en - st).sum() / (peak * span)) if peak else 0.0
    # per XCD (xcc_id): workgroups, median lifetime, last end -- a static
    # block map makes the slowest XCD's last end the kernel's end
    xcc = rec[:, 6] & 0xF
    work = blk >= nls
    res["per_xcd"] = {int(x): {"n": int((work & (xcc == x)).sum()),
                               "life_us_p50": float(np.median((en - st)[work & (xcc == x)])),
                               "last_end_us": float(en[work & (xcc == x)].max())}
                      for x in range(8) if (work & (xcc == x)).any()}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npy")
    ap.add_argument("--nls", type=int, default=0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    res = analyse(np.load(a.npy), a.nls)
    if a.json:
        print(json.dumps(res))
        return
    for k, v in res.items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    main()
