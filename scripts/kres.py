"""Per-kernel resource usage of a HIP source: python scripts/kres.py csrc/frame_td.hip [filter]
(compiles for gfx950 with the package flags and prints VGPRs / scratch / occupancy / LDS)."""
import os
import re
import subprocess
import sys
import tempfile

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-accel-ofdm-ls-mrc_amd")
src = sys.argv[1] if os.path.isabs(sys.argv[1]) else os.path.join(PKG, sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
with tempfile.TemporaryDirectory() as d:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-fno-slp-vectorize", f"-I{PKG}/build/gen", f"-I{PKG}/csrc", f"-I{PKG}/../include",
                        "-c", src, "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
cur = None
rows = {}
for ln in r.stderr.splitlines():
    m = re.search(r"remark: (.*?)\s*\[-Rpass", ln)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, d in rows.items():
    dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    short = re.sub(r"\(.*", "", dm).replace("ofdm::", "")
    if flt in short:
        print(f"{short:60s} vgpr {d.get('VGPRs', '?'):>4} scratch {d.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"occ {d.get('Occupancy [waves/SIMD]', '?')} lds {d.get('LDS Size [bytes/block]', '?')}")
if r.returncode:
    print(r.stderr[-2000:])
