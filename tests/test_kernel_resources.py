"""Every kernel of the product library runs without a private segment.

A private segment in these kernels means spilled registers, and spills on a
hot path cost 4-7 % even at two scratch accesses per antenna row (DESIGN.md
4.10: the hoisted lane index; 4.8: the generic receiver's 260-296 B), while
the segment's size alone costs nothing (the unused 416-B probe).  The
kernels form per-lane index math where it is used (lane_here / tid_here) to
stay spill-free; this test reads each kernel's .private_segment_fixed_size
from the gfx950 code objects inside lib/libofdm_lsmrc.so (llvm-objcopy,
clang-offload-bundler, llvm-readelf from /opt/rocm) and fails when any is
not 0.  CPU only: no kernel runs."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd", "lib", "libofdm_lsmrc.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TOOLS = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]


def kernel_private_segments(lib):
    """{kernel symbol: private segment bytes} of every gfx950 code object in lib."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([TOOLS[0], "--dump-section", f".hip_fatbin={fat}", lib], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", data)] + [len(data)]
        for i in range(len(starts) - 1):  # one bundle per translation unit
            b, o = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.o")
            with open(b, "wb") as fp:
                fp.write(data[starts[i]:starts[i + 1]])
            r = subprocess.run([TOOLS[1], "--unbundle", "--type=o", f"--input={b}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={o}"], capture_output=True)
            if r.returncode or not os.path.exists(o) or os.path.getsize(o) == 0:
                continue  # a host-only translation unit
            notes = subprocess.run([TOOLS[2], "--notes", o], capture_output=True, text=True, check=True).stdout
            name = None
            for ln in notes.splitlines():
                m = re.search(r"^\s+\.name:\s+(\S+)", ln)
                if m:
                    name = m.group(1)  # the kernel's .name follows its .args (keys are sorted)
                m = re.search(r"\.private_segment_fixed_size:\s+(\d+)", ln)
                if m and name:
                    out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(LIB) or not all(os.path.exists(t) for t in TOOLS),
                    reason="product library or ROCm LLVM tools absent")
def test_product_kernels_have_no_private_segment():
    seg = kernel_private_segments(LIB)
    # the receivers this round made spill-free are among them
    for k in ("k_demod_td1024", "k_mrc_td1024_hlds", "k_mrc_td2048", "k_mrc_td4096h", "k_mrc_td3072",
              "k_mrc_td6144", "k_mrc_any"):
        assert any(k in n for n in seg), f"{k} not found in the library's code objects"
    spilled = {n: v for n, v in seg.items() if v}
    assert not spilled, f"kernels with a private segment (spills): {spilled}"
    assert len(seg) >= 100
