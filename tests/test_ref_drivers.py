"""The reference's own drivers against the drop-in boundary (north_star: "the
ShMemSymBuff host ingest and cpuLS/gpuLS entry points keep their C++ API
surface so the existing rx/tx drivers can call in unchanged").

CPU (this container, where /root/reference exists; skipped elsewhere):
  * cpuLS_main.cpp, unchanged, compiles and links with the exact command of
    INTEGRATION.md section 2 (read from the file, so the document is tested);
  * oracle/build_drivers.sh builds the unchanged cpuLS_main.cpp, the
    mechanically ported gpuLS_main.cu (host/port_cuda_driver.sed) and the
    reference's own ring writer (rx_and_corr.cpp:48-60 + copy_to_shared_mem,
    64-87) into oracle/_ref/drivers/.
GPU (the binaries travel with the tree; the reference sources do not):
  rx_and_corr's writer -> ShMemSymBuff ring -> cpuLS_main / gpuLS_main ->
  Output_{cpu,gpu}.dat == golden output (reference arithmetic, tests/golden/).
"""
import glob
import os
import re
import shutil
import signal
import subprocess
import time

import numpy as np
import pytest

from helpers import GOLDEN, parity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd")
REF = "/root/reference"
DRV = os.path.join(ROOT, "oracle", "_ref", "drivers")

needs_src = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "cpuLS_main.cpp")),
                               reason="reference sources not present (GPU box)")


def integration_command(which):
    """The g++ line INTEGRATION.md section 2 gives for `which` (cpuLS_main.cpp
    or gpuLS_main.cpp), with its backslash continuations joined."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"```sh\n(.*?)```", text[text.index("## 2."):], re.S).group(1)
    joined = block.replace("\\\n", " ")
    for line in joined.splitlines():
        if line.strip().startswith("g++") and which in line:
            return line.strip()
    raise AssertionError(f"no g++ line for {which} in INTEGRATION.md section 2")


@needs_src
def test_cpuLS_main_unchanged_builds_with_integration_recipe(tmp_path):
    shutil.copy(os.path.join(REF, "cpuLS_main.cpp"), tmp_path)
    os.symlink(os.path.join(ROOT, "include"), tmp_path / "include")
    cmd = integration_command("cpuLS_main.cpp")
    env = dict(os.environ, PKG=PKG, PWD=str(tmp_path))
    r = subprocess.run(["bash", "-c", cmd], cwd=tmp_path, env=env, capture_output=True, text=True)
    assert r.returncode == 0, cmd + "\n" + r.stderr
    assert (tmp_path / "cpuLS").exists()
    # the only diagnostic is the reference's own macro redefinition
    # (cpuLS.hpp:62 `mode 1` vs cpuLS_main.cpp:35 `mode 0`)
    errs = [l for l in r.stderr.splitlines() if "error" in l]
    assert not errs, r.stderr


@needs_src
def test_ported_gpuLS_main_builds_with_integration_recipe(tmp_path):
    src = subprocess.run(["sed", "-f", os.path.join(PKG, "host", "port_cuda_driver.sed"),
                          os.path.join(REF, "gpuLS_main.cu")], capture_output=True, text=True,
                         check=True).stdout
    code = [l for l in src.splitlines() if not l.strip().startswith("//")]
    assert not [l for l in code if "cufft" in l or "cuda" in l.lower().replace("cudaen", "")], \
        "CUDA names left after the port"
    (tmp_path / "gpuLS_main.cpp").write_text(src)
    os.symlink(os.path.join(ROOT, "include"), tmp_path / "include")
    cmd = integration_command("gpuLS_main.cpp")
    env = dict(os.environ, PKG=PKG, PWD=str(tmp_path))
    r = subprocess.run(["bash", "-c", cmd], cwd=tmp_path, env=env, capture_output=True, text=True)
    assert r.returncode == 0, cmd + "\n" + r.stderr
    assert (tmp_path / "gpuLS").exists()


@needs_src
def test_build_drivers_recipe():
    r = subprocess.run(["bash", os.path.join(ROOT, "oracle", "build_drivers.sh")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    for tag in ("r4_c1024_s10", "r8_c2048_s3"):
        for exe in ("cpuLS_main", "gpuLS_main", "rx_writer"):
            assert os.access(os.path.join(DRV, f"{exe}_{tag}"), os.X_OK), (exe, tag)


def test_writer_runs_without_gpu(tmp_path):
    """The rx_and_corr writer built from the reference's own code runs on a
    host without a GPU (the ring is plain shared memory): it fills the ring
    frame after frame; a stand-in slave checks the ring content, then
    detaches, which ends the writer."""
    exe = os.path.join(DRV, "rx_writer_r4_c1024_s10")
    if not os.access(exe, os.X_OK):
        pytest.skip("oracle/_ref/drivers not built")
    z = np.load(os.path.join(GOLDEN, "cfg1_r4_c1024_s10.npz"), allow_pickle=False)
    iq = z["iq"][0]  # S x R x (C + cp)
    S, R, Cp = iq.shape
    iq.transpose(1, 0, 2).astype(np.complex64).tofile(tmp_path / "iq.bin")
    _unlink("/ofdm_refdrv_r4_c1024_s10")
    w = subprocess.Popen([exe, "iq.bin", str(int(z["prefix"]))], cwd=tmp_path,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        path = "/dev/shm/ofdm_refdrv_r4_c1024_s10"
        hdr = 12
        nbytes = hdr + S * R * 1024 * 8
        for _ in range(2000):  # writer is master: wait for its full ring
            if os.path.exists(path) and os.path.getsize(path) == nbytes:
                h = np.fromfile(path, np.int32, 3)
                if h[0] == S and h[2] == 0:  # size, writePtr wrapped after S writes
                    break
            time.sleep(0.005)
        time.sleep(0.01)  # mid-period: the frame's S writes are complete
        ring = np.fromfile(path, np.uint8)
        sym = ring[hdr:].view(np.complex64).reshape(S, R, 1024)
        np.testing.assert_array_equal(sym, iq[:, :, int(z["prefix"]):])
        hdrv = ring[:hdr].view(np.int32)
        hdrv[0] = -1  # the slave's detach (ShMemSymBuff dtor): the writer exits
        with open(path, "r+b") as f:
            f.write(hdrv.tobytes())
        out, err = w.communicate(timeout=30)
        assert w.returncode == 0, out + err
    finally:
        if w.poll() is None:
            w.kill()
        _unlink("/ofdm_refdrv_r4_c1024_s10")


def _unlink(name):
    p = "/dev/shm" + name
    if os.path.exists(p):
        os.unlink(p)


def raw_pilots(X):
    """Inverse of matrix_readX's rotation: the file content that reads as X."""
    K = X.size
    return X[(np.arange(K) - (K + 1) // 2) % K]


@pytest.mark.gpu
@pytest.mark.parametrize("reader", ["cpuLS_main", "gpuLS_main"])
@pytest.mark.parametrize("fixture,tag", [("cfg1_r4_c1024_s10", "r4_c1024_s10"),
                                         ("r8_c2048_s3_cp16", "r8_c2048_s3")])
def test_reference_drivers_end_to_end(tmp_path, reader, fixture, tag):
    """rx_and_corr.cpp's copy_to_shared_mem (writeNextSymbolNoWait, cyclic
    prefix dropped by the writer) -> ring -> the reference's cpuLS_main
    (unchanged) or gpuLS_main (mechanically ported) -> Output_*.dat."""
    wexe, rexe = (os.path.join(DRV, f"{e}_{tag}") for e in ("rx_writer", reader))
    if not (os.access(wexe, os.X_OK) and os.access(rexe, os.X_OK)):
        pytest.skip("oracle/_ref/drivers not built (build_drivers.sh runs where the reference is)")
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    iq = z["iq"][0]  # first frame: S x R x (C + cp)
    S, R, Cp = iq.shape
    C = Cp - int(z["prefix"])
    raw_pilots(z["X"]).astype(np.complex64).tofile(tmp_path / "Pilots.dat")
    iq.transpose(1, 0, 2).astype(np.complex64).tofile(tmp_path / "iq.bin")  # channel-major
    _unlink(f"/ofdm_refdrv_{tag}")
    # the reader (slave) first, spinning until the writer (master) creates the
    # ring: the NoWait writer never waits for it (rx_and_corr.cpp:83)
    r = subprocess.Popen([rexe], cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    w = None
    try:
        time.sleep(0.3)
        w = subprocess.Popen([wexe, "iq.bin", str(int(z["prefix"]))], cwd=tmp_path,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        rout, rerr = r.communicate(timeout=120)
        assert r.returncode == 0, rout + rerr
        # the radio loop runs until SIGINT (rx_and_corr.cpp:56-57, 305); the
        # unchanged cpuLS_main never deletes its ring (cpuLS_main.cpp:98), so
        # the writer is stopped the way the reference's is
        if w.poll() is None:
            w.send_signal(signal.SIGINT)
        wout, werr = w.communicate(timeout=30)
        assert w.returncode == 0, wout + werr
    finally:
        for p in (r, w):
            if p is not None and p.poll() is None:
                p.kill()
        _unlink(f"/ofdm_refdrv_{tag}")
    name = "Output_cpu.dat" if reader == "cpuLS_main" else "Output_gpu.dat"
    got = np.fromfile(tmp_path / name, np.complex64).reshape(S - 1, C - 1)
    parity(got, z["out"][0])
