"""Per-kernel-variant table of the SQ counters collected by scripts/experiments/gpu_sq_ab.sh.
usage: python scripts/experiments/sq_table.py gpurun_out/sqab_<tag> [kernel-name filter, default k_mrc_td]
WAVE/WAIT/ACTIVE counters are quad-cycles (MI355X_MICROARCH.md); ratios are
per wave lifetime (SQ_WAVE_CYCLES)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "k_mrc_td"
val = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fp:
        for row in csv.DictReader(fp):
            k = row["Kernel_Name"]
            if flt not in k:
                continue
            k = k.split("(")[0].replace("void ", "").split("::")[-1]
            val[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, c in sorted(val.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    w = m.get("SQ_WAVES", 1.0)
    print(k)
    print("  per wave: VALU %.0f  LDS %.0f  SALU %.0f  VMEM_RD %.0f" % (
        m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_LDS", 0) / w, m.get("SQ_INSTS_SALU", 0) / w,
        m.get("SQ_INSTS_VMEM_RD", 0) / w))
    print("  of wave cycles: wait_any %.2f  wait_inst_any %.2f  wait_inst_lds %.2f  active_any %.2f  "
          "active_valu %.2f  active_lds %.2f  active_vmem %.2f  active_sca %.2f" % tuple(
              m.get(n, 0) / wc for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                                         "SQ_ACTIVE_INST_SCA")))
    print("  LDS bank conflict cycles / LDS inst: %.2f   busy cycles %.3g   wave cycles/wave %.3g" % (
        m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_INSTS_LDS", 1), 1), m.get("SQ_BUSY_CYCLES", 0), wc / w))
