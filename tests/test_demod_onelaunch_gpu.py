"""The one-launch frame demod (k_demod_td1024: estimator workgroups publish
each frame's estimate to the MRC workgroups of the same grid through the
workspace's flag words; k_demod_td2048 / 4096 in the A/B build only).
ofdm_frame_demod at C = 1024 takes this path;
these tests hold it to the two-launch flow (ofdm_frame_estimate +
ofdm_frame_combine, itself tested against the oracle in test_gpu_parity.py)
and to the oracle, on shapes with straddling workgroups (8 symbols spanning
two frames) and tail waves, on a reused workspace with new data (the flags
of the previous launch must not release the next one), and with the bounded
wait forced to expire (A/B build: every MRC workgroup estimates its frames
itself).  Tolerance: helpers.RTOL.  At C = 1024 the estimator sums |H|^2
over antennas in the 8-wave order (rows w, w+8, ... per wave, then waves in
order), the two-launch LS in its own wave order, so the outputs agree to
rounding, not bit for bit; at C = 2048 / 4096 (A/B build) the estimator is
the LS kernel's own code and the outputs are bit-identical."""
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import RTOL, parity

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def pilots(dev, K, seed=5):
    import torch
    rng = np.random.default_rng(seed)
    a = np.float32(0.70710678)
    X = (rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)
    return torch.from_numpy(X).to(dev)


def two_launch(ofdm, iq, X, prefix):
    F, S, R, Cp = iq.shape
    ws = ofdm.workspace(F, S, R, Cp - prefix, iq.device)
    out = ofdm.c64((F, S - 1, Cp - prefix - 1), iq.device)
    ofdm.frame_estimate(iq, X, prefix, ws)
    ofdm.frame_combine(iq, prefix, ws, out)
    return host(out)


# (C, F, S, R, prefix): C=1024 100 x 101 x 16 is BASELINE configs[1]; S - 1
# = 100 and 6 symbols per frame put workgroups across frame boundaries;
# 7 x 3 = 21 symbols leaves tail waves in the last workgroup; R = 1 and R = 9
# leave estimator waves without rows / with one extra row.  C = 4096
# workgroups are frame-aligned (4 symbols): S = 7 leaves tail pairs.
@pytest.mark.parametrize("C,F,S,R,prefix", [(1024, 100, 101, 16, 0), (1024, 7, 4, 1, 0), (1024, 5, 7, 9, 8),
                                            (1024, 3, 101, 64, 72), (1024, 1, 2, 4, 0), (1024, 40, 13, 16, 0)])
def test_one_launch_matches_two_launch(ofdm, dev, C, F, S, R, prefix):
    X = pilots(dev, C - 1)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=F * 1000 + S * 10 + R, noise_std=0.01)
    got = host(ofdm.frame_demod(iq, X, prefix))
    ref = two_launch(ofdm, iq, X, prefix)
    parity(got, ref)
    if R >= 16:  # enough receive diversity for error-free QPSK at sigma = 0.01 (R = 1 fades)
        assert int(ofdm.count_symbol_errors(ofdm.frame_demod(iq, X, prefix), S,
                                            seed=F * 1000 + S * 10 + R).item()) == 0


@pytest.mark.parametrize("C", [1024])
def test_one_launch_vs_oracle(ofdm, oracle, dev, C):
    """First and last frame of a straddling batch against the C oracle."""
    F, S, R, prefix = 6, 7, 5, 8
    X = pilots(dev, C - 1, seed=9)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=77, noise_std=0.02)
    out = host(ofdm.frame_demod(iq, X, prefix))
    xs = host(X)
    for f in (0, F - 1):
        ref, _, _ = oracle.frame_demod(host(iq[f]), xs, prefix)
        parity(out[f], ref)


@pytest.mark.parametrize("C", [1024])
def test_reused_workspace_new_data(ofdm, dev, C):
    """Launch N+1 on the workspace of launch N with other frames: its MRC
    workgroups must wait for the new estimates (new epoch), not read the old
    ones the flags of launch N still vouch for."""
    F, S, R = 24, 21, 16
    X = pilots(dev, C - 1)
    a = ofdm.synth_frames(F, S, R, C, X, seed=1, noise_std=0.01)
    b = ofdm.synth_frames(F, S, R, C, X, seed=2, noise_std=0.01)
    ws = ofdm.workspace(F, S, R, C, dev)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    for rep in range(3):
        ofdm.frame_demod(a, X, 0, ws=ws, out=out)
        got_a = host(out)
        ofdm.frame_demod(b, X, 0, ws=ws, out=out)
        got_b = host(out)
        if rep == 0:
            ref_a, ref_b = two_launch(ofdm, a, X, 0), two_launch(ofdm, b, X, 0)
        parity(got_a, ref_a)
        parity(got_b, ref_b)
    # the estimate left in the workspace is b's, in the fused lane order
    e = ofdm.frame_export_estimate(ws, F, S, R, C, frame=F - 1)
    ws2 = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_estimate(b, X, 0, ws2)
    e2 = ofdm.frame_export_estimate(ws2, F, S, R, C, frame=F - 1)
    parity(host(e[0]), host(e2[0]))
    parity(host(e[1]), host(e2[1]), rtol=RTOL)


def test_one_launch_under_uneven_load(ofdm, dev):
    """The hand-off under uneven load (cdna_hip_programming.md Guideline 16:
    test with the GPU busy elsewhere, consumers L1-warm): frame_demod runs
    repeatedly on one stream while another stream streams a large
    elementwise kernel, on a reused workspace, with the batch alternating
    between two inputs; every output must match its two-launch reference."""
    import torch
    F, S, R, C = 60, 13, 16, 1024
    X = pilots(dev, C - 1)
    a = ofdm.synth_frames(F, S, R, C, X, seed=21, noise_std=0.01)
    b = ofdm.synth_frames(F, S, R, C, X, seed=22, noise_std=0.01)
    ref = {0: two_launch(ofdm, a, X, 0), 1: two_launch(ofdm, b, X, 0)}
    ws = ofdm.workspace(F, S, R, C, dev)
    outs = [ofdm.c64((F, S - 1, C - 1), dev) for _ in range(6)]
    hog = torch.empty(1 << 28, dtype=torch.float32, device=dev).uniform_()
    busy, work = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(busy):
        for _ in range(6):
            hog.mul_(1.0000001).add_(1e-7)
    for i, o in enumerate(outs):
        ofdm.frame_demod(a if i % 2 == 0 else b, X, 0, ws=ws, out=o, stream=work)
        if i == 2:
            with torch.cuda.stream(busy):
                hog.mul_(0.9999999)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        parity(host(o), ref[i % 2])


def test_graph_capture_takes_two_launches(ofdm, dev):
    """Under stream capture ofdm_frame_demod uses the two launches (a frozen
    epoch would let a replay read stale estimates); the replayed graph then
    demodulates new data written into the captured input buffer."""
    import torch
    F, S, R, C = 8, 11, 16, 1024
    X = pilots(dev, C - 1)
    a = ofdm.synth_frames(F, S, R, C, X, seed=3, noise_std=0.01)
    b = ofdm.synth_frames(F, S, R, C, X, seed=4, noise_std=0.01)
    iq = a.clone()
    ws = ofdm.workspace(F, S, R, C, dev)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    st = torch.cuda.Stream()
    ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)  # warm (outside capture)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
    iq.copy_(b)
    g.replay()
    parity(host(out), two_launch(ofdm, b, X, 0))
    iq.copy_(a)
    g.replay()
    parity(host(out), two_launch(ofdm, a, X, 0))


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd", "lib",
                                                    "libofdm_lsmrc_ab.so")),
                    reason="A/B build (make -C gpu-accel-ofdm-ls-mrc_amd ab) not present")
@pytest.mark.parametrize("C", [1024, 2048, 4096])
def test_bounded_wait_fallback_ab_build(C):
    """OFDM_AB_DEMOD_SPIN=0: no MRC workgroup waits for a flag; each
    estimates its frame(s) itself.  Same outputs as the normal path, and the
    one launch agrees with two (run in a child process on the A/B library)."""
    code = r"""
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(sys.argv[1], "gpu-accel-ofdm-ls-mrc_amd"))
import ofdm_lsmrc as ofdm
F, S, R, C = 9, 13, 16, int(sys.argv[2])
a = np.float32(0.70710678); rng = np.random.default_rng(5)
X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)).cuda()
iq = ofdm.synth_frames(F, S, R, C, X, seed=11, noise_std=0.01)
os.environ["OFDM_AB_DEMOD_FUSED"] = "0"
two = ofdm.frame_demod(iq, X).cpu().numpy()
os.environ.pop("OFDM_AB_DEMOD_FUSED")
ref = ofdm.frame_demod(iq, X).cpu().numpy()
os.environ["OFDM_AB_DEMOD_SPIN"] = "0"
got = ofdm.frame_demod(iq, X).cpu().numpy()
d = np.abs(got - ref).max() / np.abs(ref).max()
d2 = np.abs(ref - two).max() / np.abs(two).max()
print("maxrel fallback vs one launch", d, "one launch vs two", d2)
ok = d <= 1e-6 and d2 <= 1e-5 and (C == 1024 or d2 == 0)
sys.exit(0 if ok else 1)
"""
    # C = 2048 / 4096: the one-launch kernels of the A/B build (OFDM_AB_DEMOD_WIDE;
    # no faster than two launches, not in the product), bit-identical to two launches
    env = dict(os.environ, OFDM_LSMRC_LIB="ab", OFDM_AB_DEMOD_WIDE="1")
    p = subprocess.run([sys.executable, "-c", code, ROOT, str(C)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
