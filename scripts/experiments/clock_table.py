"""Mean effective clock per MRC kernel variant from a rocprofv3 run with
--kernel-trace and --pmc GRBM_GUI_ACTIVE: cycles / 8 / (end - start) -- the
counter is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
cyc = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_mrc_td" in row["Kernel_Name"]:
            cyc[row.get("Dispatch_Id") or row.get("Correlation_Id")].append(
                (row["Kernel_Name"].split("(")[0].split("::")[-1], float(row["Counter_Value"])))
dur = {}
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_mrc_td" in row["Kernel_Name"]:
            dur[row.get("Dispatch_Id") or row.get("Correlation_Id")] = (
                float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
agg = defaultdict(list)
for k, v in cyc.items():
    if k in dur:
        name = v[0][0]
        agg[name].append((sum(x[1] for x in v), dur[k]))
for name, v in agg.items():
    mhz = [c / 8 / ns * 1e3 for c, ns in v]
    print(f"{name}: {len(v)} dispatches, {sum(ns for _, ns in v) / len(v) / 1e6:.3f} ms avg, "
          f"clock {sum(mhz) / len(mhz):.0f} MHz (min {min(mhz):.0f}, max {max(mhz):.0f})")
