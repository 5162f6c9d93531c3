"""End-to-end through the drop-in boundary on the GPU: a writer process
(master, like rx_and_corr.cpp) pushes IQ symbols through the ShMemSymBuff
shared-memory ring; a reader process runs one of the reference's receiver
flows written against this package's headers (cpuLS.hpp free functions,
gpuLS per-symbol with a host or a device staging buffer, gpuLS frame, and
the pipelined multi-frame gpuLS::demodFrames); its Output_*.dat must match
the golden output computed by the reference's own arithmetic
(tests/golden/)."""
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN, parity

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd")
CPP = os.path.join(ROOT, "tests", "cpp")


def raw_pilots(X):
    """Inverse of matrix_readX's rotation: the file content that reads as X."""
    K = X.size
    return X[(np.arange(K) - (K + 1) // 2) % K]


def build(tmp, name, R, C, prefix, S, shm):
    exe = os.path.join(tmp, name)
    cmd = ["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           f"-I{PKG}/host", f"-I{ROOT}/include", f"-DnumOfRows={R}", f"-Ddimension={C}",
           f"-Dprefix={prefix}", f"-DlenOfBuffer={S}", f"-DshmemID=\"{shm}\"",
           os.path.join(CPP, name + ".cpp"), "-o", exe, f"-L{PKG}/lib", "-lofdm_lsmrc",
           f"-Wl,-rpath,{PKG}/lib", "-L/opt/rocm/lib", "-lamdhip64", "-lrt"]
    subprocess.run(cmd, check=True)
    return exe


@pytest.mark.parametrize("fixture,flow", [("cfg1_r4_c1024_s10", "cpuls"),
                                          ("cfg1_r4_c1024_s10", "symbol"),
                                          ("cfg1_r4_c1024_s10", "symbolcuda"),
                                          ("r8_c2048_s3_cp16", "symbolcuda"),
                                          ("cfg1_r4_c1024_s10", "frame"),
                                          ("r8_c2048_s3_cp16", "symbol"),
                                          ("r8_c2048_s3_cp16", "cpuls"),
                                          ("r4_c256_s5_cp32", "frame"),
                                          ("r8_c2048_s3_cp16", "frame"),
                                          ("r16_c1024_s4_2frames", "frame"),
                                          ("cfg1_r4_c1024_s10", "symboledit"),
                                          ("r8_c2048_s3_cp16", "symboledit")])
def test_ring_to_output_file(tmp_path, fixture, flow):
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    iq = z["iq"][0]  # first frame: S x R x (C + prefix)
    S, R, Cp = iq.shape
    prefix = int(z["prefix"])
    C = Cp - prefix
    tmp = str(tmp_path)
    raw_pilots(z["X"]).astype(np.complex64).tofile(os.path.join(tmp, "Pilots.dat"))
    iq.astype(np.complex64).tofile(os.path.join(tmp, "iq.bin"))
    shm = f"/ofdm_e2e_{os.getpid()}_{flow}_{C}"
    writer = build(tmp, "e2e_writer", R, C, prefix, S, shm)
    reader = build(tmp, "e2e_reader", R, C, prefix, S, shm)
    w = subprocess.Popen([writer, "iq.bin"], cwd=tmp, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        r = subprocess.run([reader, flow], cwd=tmp, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        out, err = w.communicate(timeout=60)
        assert w.returncode == 0, out + err
    finally:
        if w.poll() is None:
            w.kill()
    name = "Output_cpu.dat" if flow == "cpuls" else "Output_gpu.dat"
    got = np.fromfile(os.path.join(tmp, name), np.complex64).reshape(S - 1, C - 1)
    if flow == "symboledit":
        # an in-place edit of Hsqrd after firstVector is seen by
        # demodOneSymbol (gpuLS.cu:410-473 reads it for every symbol), not
        # masked by the fused path's kept estimate
        parity(got, z["out"][0] / 2)
        return
    parity(got, z["out"][0])
    if flow != "cpuls":  # the LS estimate the gpuLS flow leaves in its Hconj / Hsqrd arguments
        H = np.fromfile(os.path.join(tmp, "Hconj_gpu.dat"), np.complex64).reshape(R, C - 1)
        P = np.fromfile(os.path.join(tmp, "Hsqrd_gpu.dat"), np.float32)
        parity(H, z["H"][0])
        parity(P, z["P"][0])


@pytest.mark.parametrize("fixture,repeat,chunk,depth", [("r16_c1024_s4_2frames", 1, 4, 3),
                                                        ("r4_c256_s5_cp32", 1, 1, 1),
                                                        ("r3_c64_s4_odd_antennas", 7, 3, 2),
                                                        ("r16_c1024_s4_2frames", 20, 4, 3)])
def test_ring_frames_pipelined(tmp_path, fixture, repeat, chunk, depth):
    """gpuLS::demodFrames: every frame of the fixture, pushed `repeat` times
    through a one-frame ring, read by the pipelined bulk reader into the
    ofdm_pipeline slots (ring and pipeline wrap many times)."""
    z = np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False)
    iq = z["iq"]  # F x S x R x (C + prefix)
    F, S, R, Cp = iq.shape
    prefix = int(z["prefix"])
    C = Cp - prefix
    tmp = str(tmp_path)
    raw_pilots(z["X"]).astype(np.complex64).tofile(os.path.join(tmp, "Pilots.dat"))
    iq.astype(np.complex64).tofile(os.path.join(tmp, "iq.bin"))
    shm = f"/ofdm_e2e_{os.getpid()}_frames_{C}_{repeat}"
    writer = build(tmp, "e2e_writer", R, C, prefix, S, shm)
    reader = build(tmp, "e2e_reader", R, C, prefix, S, shm)
    w = subprocess.Popen([writer, "iq.bin", str(repeat)], cwd=tmp, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    nframes = F * repeat
    try:
        r = subprocess.run([reader, "frames", str(nframes), str(chunk), str(depth)], cwd=tmp,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        out, err = w.communicate(timeout=60)
        assert w.returncode == 0, out + err
    finally:
        if w.poll() is None:
            w.kill()
    print(r.stdout.strip())
    got = np.fromfile(os.path.join(tmp, "Output_gpu.dat"), np.complex64)
    got = got.reshape(nframes, S - 1, C - 1)
    parity(got, np.tile(z["out"], (repeat, 1, 1)))
