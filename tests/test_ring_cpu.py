"""CPU tests of the host boundary: the ShMemSymBuff ring between two
processes (writer = master, reader = slave), built at -O2 where the
reference's plain-int ring loses symbols, plus a compile check
of the cpuLS.hpp / gpuLS.hpp mirrors with the host compiler."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd", "host")
CPP = os.path.join(ROOT, "tests", "cpp")


def build_ring(tmp_path, L, prefix, san):
    exe = tmp_path / f"ring_{L}_{prefix}_{int(san)}"
    cmd = ["g++", "-O2", "-std=c++17", f"-I{HOST}", "-DnumOfRows=2", "-Ddimension=16",
           f"-Dprefix={prefix}", f"-DlenOfBuffer={L}",
           f"-DshmemID=\"/ofdm_ring_{os.getpid()}_{L}_{prefix}_{int(san)}\"",
           os.path.join(CPP, "ring_test.cpp"), "-o", str(exe), "-lrt"]
    if san:
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    subprocess.run(cmd, check=True)
    return exe


@pytest.mark.parametrize("L,prefix,san", [(4, 0, False), (11, 3, False), (3, 0, True),
                                          (101, 0, False)])
def test_ring_two_process_with_wait(tmp_path, L, prefix, san):
    exe = build_ring(tmp_path, L, prefix, san)
    r = subprocess.run([str(exe), str(5 * L + 2), "wait"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


def test_ring_two_process_nowait_paced(tmp_path):
    # the NoWait writer never blocks (rx_and_corr.cpp:83); paced slower than
    # the reader it must still deliver every symbol in order
    exe = build_ring(tmp_path, 8, 2, False)
    r = subprocess.run([str(exe), "40", "nowait"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_host_mirror_headers_compile(tmp_path):
    """cpuLS.hpp and gpuLS.hpp compile with the host compiler against the HIP
    runtime headers and link against the C ABI library."""
    src = tmp_path / "t.cpp"
    src.write_text('#include "cpuLS.hpp"\n#include "gpuLS.hpp"\n'
                   'int main(){ gpuLS *g = nullptr; (void)g; complexF c{1,2}; (void)c;'
                   ' return 0; }\n')
    lib = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{HOST}", f"-I{os.path.join(ROOT, 'include')}", str(src),
                    "-o", str(tmp_path / "t"), f"-L{lib}", "-lofdm_lsmrc",
                    "-L/opt/rocm/lib", "-lamdhip64", "-lrt"], check=True)


@pytest.mark.parametrize("L,prefix,n,mode", [(5, 3, 40, "wait"), (101, 0, 250, "wait"), (8, 2, 30, "nowait")])
def test_ring_protocol_under_tsan(tmp_path, L, prefix, n, mode):
    """Writer and reader threads on ONE ring object under ThreadSanitizer
    (the reference's plain-int ring races; here the slots and
    indices must be ordered by the acquire/release protocol)."""
    exe = tmp_path / "ring_tsan"
    subprocess.run(["g++", "-O1", "-g", "-fsanitize=thread", "-std=c++17", f"-I{HOST}", "-DnumOfRows=2",
                    "-Ddimension=16", f"-Dprefix={prefix}", f"-DlenOfBuffer={L}",
                    f"-DshmemID=\"/ofdm_tsan_{os.getpid()}_{L}_{mode}\"", os.path.join(CPP, "ring_tsan.cpp"),
                    "-o", str(exe), "-lrt"], check=True)
    r = subprocess.run([str(exe), str(n), mode], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ThreadSanitizer" not in r.stderr, r.stderr
    assert r.stdout.startswith("ok")
