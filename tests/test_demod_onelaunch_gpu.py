"""The one-launch frame demod (k_demod_td1024: estimator workgroups publish
each frame's estimate to the MRC workgroups of the same grid through the
workspace's flag words).
ofdm_frame_demod at C = 1024 takes this path;
these tests hold it to the two-launch flow (ofdm_frame_estimate +
ofdm_frame_combine, itself tested against the oracle in test_gpu_parity.py)
and to the oracle, on shapes with straddling workgroups (8 symbols spanning
two frames) and tail waves, on a reused workspace with new data (the flags
of the previous launch must not release the next one), and with the bounded
wait forced to expire (ofdm_frame_demod_ex spin_ticks = 0: every MRC
workgroup estimates its frames itself).  Tolerance: helpers.RTOL.  The
estimator sums |H|^2 over antennas in the 8-wave order (rows w, w+8, ...
per wave, then waves in order), the two-launch LS in its own wave order, so
the outputs agree to rounding, not bit for bit."""
import os

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


def torch_index(idx, device):
    import torch
    return torch.as_tensor(idx, device=device)


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
# Batches of more than 512 workgroups' blocks take work tickets: 60 x 101 x
# 9 (every ticketed block split into two half units, 5 + 4 rows per wave)
# and 150 x 101 x 3 (whole tickets, then half units of 2 + 1 rows).
@pytest.mark.parametrize("C,F,S,R,prefix", [(1024, 100, 101, 16, 0), (1024, 7, 4, 1, 0), (1024, 5, 7, 9, 8),
                                            (1024, 3, 101, 64, 72), (1024, 1, 2, 4, 0), (1024, 40, 13, 16, 0),
                                            (1024, 60, 101, 9, 8), (1024, 150, 101, 3, 0)])
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


@pytest.mark.parametrize("F,S,R", [(9, 13, 16), (3, 101, 64), (20, 5, 4), (60, 101, 4)])
def test_bounded_wait_fallback(ofdm, dev, F, S, R):
    """ofdm_frame_demod_ex with spin_ticks = 0: no MRC workgroup waits for a
    flag; each estimates the frame(s) it reads itself, through the same
    hlds_ls_frame call site as the estimator workgroups.  The output must be
    bit-identical to the default one-launch path's (same code, same bytes),
    and within rounding of the two-launch flow (different FFT kernels)."""
    import torch
    C = 1024
    rng = np.random.default_rng(5 + R)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=11, noise_std=0.01)
    ref = ofdm.frame_demod(iq, X)
    got = ofdm.frame_demod(iq, X, spin_ticks=0)
    two = ofdm.frame_demod(iq, X, flow=ofdm.FLOW_TWO_LAUNCH)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    parity(host(ref), host(two), rtol=1e-6)
    assert int(ofdm.count_symbol_errors(got, S, seed=11).item()) == 0


def test_frame_demod_ex_rejects_unknown_flow(ofdm, dev):
    import torch
    X = torch.ones(1023, dtype=torch.complex64, device=dev)
    iq = torch.zeros((1, 2, 1, 1024), dtype=torch.complex64, device=dev)
    with pytest.raises(ofdm.OfdmError, match="flow=7"):
        ofdm.frame_demod(iq, X, flow=7)


def test_work_tickets_reused_workspace(ofdm, dev):
    """Work tickets (wave_fft1024.hpp take_unit): a batch large enough for
    ticketed blocks and half units, demodulated 4 times in turn with another
    batch on ONE workspace -- every launch claims the counters the previous
    launch left (tagged counts); every output must match its two-launch
    reference, and a repeat must be bit-identical (the schedule changes
    which workgroup takes a block, never the block's arithmetic)."""
    import torch
    F, S, R, C = 60, 101, 4, 1024
    X = pilots(dev, C - 1)
    a = ofdm.synth_frames(F, S, R, C, X, seed=31, noise_std=0.01)
    b = ofdm.synth_frames(F, S, R, C, X, seed=32, noise_std=0.01)
    ref = {0: two_launch(ofdm, a, X, 0), 1: two_launch(ofdm, b, X, 0)}
    ws = ofdm.workspace(F, S, R, C, dev)
    first = {}
    for i in range(8):
        o = ofdm.frame_demod(a if i % 2 == 0 else b, X, 0, ws=ws)
        parity(host(o), ref[i % 2])
        if i < 2:
            first[i] = o
        else:
            assert torch.equal(o, first[i % 2])


@pytest.mark.parametrize("C,F,R", [(2048, 40, 4), (4096, 16, 4)])
def test_work_tickets_wide_receivers_vs_freq_path(ofdm, dev, C, F, R):
    """The C = 2048 / 4096 receivers with work tickets active (more blocks
    than the static first round) against the frequency-domain LS + MRC on
    the same frames (fft_rows, then ofdm_frame_demod_freq: other kernels,
    pinned to the oracle in test_gpu_parity.py)."""
    S = 101
    X = pilots(dev, C - 1, seed=C)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=C + F, noise_std=0.01)
    got = host(ofdm.frame_demod(iq, X, 0))
    Y = ofdm.fft_rows(iq.clone())
    ref = host(ofdm.frame_demod_freq(Y, X))
    parity(got, ref)


@pytest.mark.parametrize("F,R", [(41, 2), (52, 2), (66, 2), (100, 2), (131, 2), (300, 2), (60, 5), (100, 4), (45, 7)])
def test_work_tickets_cover_every_unit(ofdm, dev, F, R):
    """Batch sizes around and beyond the static first round (512 blocks):
    every ticketed block and half unit must be processed exactly once (a
    grid smaller than the unit count would leave outputs unwritten: the
    output buffer is NaN-filled first, so a missed unit fails the finite
    check in parity).  R = 5 / 7 give half units of uneven row counts."""
    import torch
    S, C = 101, 1024
    X = pilots(dev, C - 1, seed=F)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=F, noise_std=0.01)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    out.fill_(float("nan"))
    ofdm.frame_demod(iq, X, 0, out=out)
    parity(host(out), two_launch(ofdm, iq, X, 0))


@pytest.mark.parametrize("C,F,R", [(2048, 64, 4), (4096, 16, 4)])
def test_graph_capture_ticketed_receivers(ofdm, dev, C, F, R):
    """The work-ticketed C = 2048 / 4096 receivers captured into a graph:
    the launch's tag is frozen in the graph, so every replay counts behind a
    zeroing kernel node of its own; replays after the first, and eager launches on the same
    workspace in between, still process every unit (outputs NaN-filled
    before each run; bit-identical to eager launches on a fresh workspace)."""
    import torch
    S = 101
    X = pilots(dev, C - 1, seed=C + 1)
    src = [ofdm.synth_frames(F, S, R, C, X, seed=C + k, noise_std=0.01) for k in (1, 2)]
    ref = [ofdm.frame_demod(a, X, 0) for a in src]
    torch.cuda.synchronize()
    iq = src[0].clone()
    ws = ofdm.workspace(F, S, R, C, dev)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    eager = ofdm.c64((F, S - 1, C - 1), dev)
    st = torch.cuda.Stream()
    ofdm.frame_demod(iq, X, 0, ws=ws, out=eager, stream=st)  # warm, outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        ofdm.frame_demod(iq, X, 0, ws=ws, out=out, stream=st)
    for k in (1, 0, 1, 1, 0):
        iq.copy_(src[k])
        out.fill_(float("nan"))
        eager.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref[k])
        with torch.cuda.stream(st):
            ofdm.frame_demod(iq, X, 0, ws=ws, out=eager, stream=st)
        torch.cuda.synchronize()
        assert torch.equal(eager, ref[k])


@pytest.mark.parametrize("C,Fbig,Fsmall", [(1024, 100, 60), (4096, 16, 12)])
def test_work_tickets_workspace_shared_by_two_geometries(ofdm, dev, C, Fbig, Fsmall):
    """One workspace (sized for the larger batch) used in turn by batches of
    two sizes: the work-ticket counters follow the estimate, at an offset that
    depends on the batch, and the smaller batch's counters lie inside the
    larger batch's estimate, so a call with the other geometry meets
    estimate bytes there and must claim them afresh (NaN-filled outputs;
    bit-identical to fresh workspaces)."""
    import torch
    S, R = 101, 2
    X = pilots(dev, C - 1, seed=7)
    big = ofdm.synth_frames(Fbig, S, R, C, X, seed=71, noise_std=0.01)
    small = ofdm.synth_frames(Fsmall, S, R, C, X, seed=72, noise_std=0.01)
    ref = [ofdm.frame_demod(big, X, 0), ofdm.frame_demod(small, X, 0)]
    ws = ofdm.workspace(Fbig, S, R, C, dev)
    for k in (0, 1, 0, 1, 1, 0):
        iq = (big, small)[k]
        out = ofdm.c64((iq.shape[0], S - 1, C - 1), dev)
        out.fill_(float("nan"))
        ofdm.frame_demod(iq, X, 0, ws=ws, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref[k])


def test_two_streams_two_workspaces_concurrently(ofdm, dev):
    """Two batches on two streams with a workspace each, enqueued in turn
    without host synchronisation (the one-launch kernels may run at the same
    time: each one's flags, epochs and work-ticket counters are its own);
    every output equals the serial run's (NaN-filled outputs)."""
    import torch
    S, R, C = 101, 4, 1024
    X = pilots(dev, C - 1, seed=9)
    iqs = [ofdm.synth_frames(F, S, R, C, X, seed=90 + F, noise_std=0.01) for F in (70, 45)]
    ref = [ofdm.frame_demod(iq, X, 0) for iq in iqs]
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    wss = [ofdm.workspace(iq.shape[0], S, R, C, dev) for iq in iqs]
    outs = [[ofdm.c64((iq.shape[0], S - 1, C - 1), dev) for _ in range(3)] for iq in iqs]
    for o in outs:
        for t in o:
            t.fill_(float("nan"))
    torch.cuda.synchronize()
    for rep in range(3):
        for i in (0, 1):
            ofdm.frame_demod(iqs[i], X, 0, ws=wss[i], out=outs[i][rep], stream=sts[i])
    torch.cuda.synchronize()
    for i in (0, 1):
        for rep in range(3):
            assert torch.equal(outs[i][rep], ref[i]), (i, rep)


@pytest.mark.parametrize("C,F,S,R", [(1024, 20000, 3, 1), (4096, 3000, 2, 1), (2048, 4000, 3, 1)])
def test_many_small_frames(ofdm, oracle, dev, C, F, S, R):
    """Batches of many tiny frames (one antenna, one or two data symbols):
    thousands of estimator workgroups ahead of the receivers at C = 1024,
    blocks of one symbol and tail pairs at C = 4096, far more ticketed blocks
    than resident workgroups; equal to the two-launch flow within rounding.
    Element-wise bound 2e-3: with ONE antenna the output is Y / H per bin, and
    over millions of Rayleigh-faded bins some |H| sit 100-1000x below their
    rms, where the two flows' float32 FFTs (different twiddle schemes) differ
    by their ~1e-7 absolute error divided by that |H|; the norm-relative
    bound stays helpers.RTOL and every output must be written (NaN-filled).
    Measured (profiles/r5/r5al_r1_conditioning.txt): 133 of 41 M elements
    above 1e-5, at |ref| 3-17x the rms, where both flows sit 1e-5..9e-5 from
    the float64 oracle alike.  A 64-frame sample is also checked against the
    oracle itself."""
    X = pilots(dev, C - 1, seed=C + F)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=F, noise_std=0.01)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    out.fill_(float("nan"))
    ofdm.frame_demod(iq, X, 0, out=out)
    got = host(out)
    parity(got, two_launch(ofdm, iq, X, 0), erel_tol=2e-3)
    # parity evidence, not only self-consistency (VERDICT r5 "weak" 1): 64
    # frames spread over the batch (first and last included) against the
    # oracle's float64 FFT + LS + MRC; element-wise bound 2e-4 for the faded
    # single-antenna bins (worst measured 8.8e-5, r5al_r1_conditioning.txt),
    # norm-relative helpers.RTOL
    idx = np.unique(np.linspace(0, F - 1, 64).astype(int))
    ref = oracle.frames_demod(iq[torch_index(idx, iq.device)].cpu().numpy(), host(X))
    parity(got[idx], ref, erel_tol=2e-4)


def ticket_words(ws, F, R, C):
    """The workspace's work-ticket counters (capi.cpp carve: Hc [F][R][C],
    P [F][C] and one flag word per frame, each padded to 256 B, then 8
    counters 128 B apart) as int64 words."""
    import torch
    up = lambda x: (x + 255) // 256 * 256
    off = up(F * R * C * 8) + up(F * C * 4) + up(F * 8)
    return ws[off:off + 1024].view(torch.int64)


@pytest.mark.parametrize("C,F,R", [(1024, 150, 3), (2048, 40, 4), (4096, 16, 4)])
def test_work_tickets_garbage_counters(ofdm, dev, C, F, R):
    """the ticket area of a workspace the registry knows
    (filled by an earlier demod, never released) overwritten with all-ones
    words, then small and large positive counts, then random bytes, before
    each ofdm_frame_demod: every word is claimed afresh by its tag, so every
    unit is processed (NaN-filled output) and the output is bit-identical to
    a fresh workspace's; no device fault is reported.  (Before round 6 a
    positive stale count skipped units and a negative one faulted at C =
    4096: gpurun_out/r5t/old.log.)"""
    import torch
    S = 101
    X = pilots(dev, C - 1, seed=C + 3)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=C + 33, noise_std=0.01)
    ref = ofdm.frame_demod(iq, X, 0)
    ws = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_demod(iq, X, 0, ws=ws)
    torch.cuda.synchronize()
    words = ticket_words(ws, F, R, C)
    g = torch.Generator(device="cpu").manual_seed(C)
    for fill in (-1, 3, 1 << 20, (7 << 32) | 5, None):
        if fill is None:
            words.copy_(torch.randint(-(1 << 62), 1 << 62, words.shape, generator=g))
        else:
            words.fill_(fill)
        out = ofdm.c64((F, S - 1, C - 1), dev)
        out.fill_(float("nan"))
        ofdm.frame_demod(iq, X, 0, ws=ws, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), fill
    ofdm.device_status()


@pytest.mark.parametrize("C,Fs", [(2048, 40), (4096, 16)])
def test_work_tickets_after_freq_estimate_of_other_geometry(ofdm, dev, C, Fs):
    """ofdm_frame_demod at a small batch, then
    ofdm_frame_demod_freq at a batch twice as large on the same workspace
    (its estimate covers the small batch's counters; no ticketed launch sees
    it), then the small ofdm_frame_demod again: its counters hold estimate
    bytes and must be claimed afresh (NaN-filled output, bit-identical to a
    fresh workspace)."""
    import torch
    S, R = 101, 2
    Fb = 2 * Fs
    X = pilots(dev, C - 1, seed=C + 5)
    small = ofdm.synth_frames(Fs, S, R, C, X, seed=C + 51, noise_std=0.01)
    big_td = ofdm.synth_frames(Fb, S, R, C, X, seed=C + 52, noise_std=0.01)
    big = ofdm.fft_rows(big_td.clone())
    del big_td
    ref = ofdm.frame_demod(small, X, 0)
    ref_big = ofdm.frame_demod_freq(big, X)
    ws = ofdm.workspace(Fb, S, R, C, dev)
    for k in range(2):
        out = ofdm.c64((Fs, S - 1, C - 1), dev)
        out.fill_(float("nan"))
        ofdm.frame_demod(small, X, 0, ws=ws, out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), k
        ob = ofdm.frame_demod_freq(big, X, ws=ws)
        torch.cuda.synchronize()
        assert torch.equal(ob, ref_big)
    ofdm.device_status()


def test_work_tickets_one_workspace_two_streams(ofdm, dev):
    """one estimate read by ofdm_frame_combine on two
    streams at once -- against the header's one-launch-at-a-time rule for a
    workspace.  Tagged counters make the overlap safe or loud: every output
    is complete and equal to the serial one, or the device status reports
    the overlap (OFDM_E_DEVICE); never a silently incomplete output."""
    import torch
    C, F, S, R = 4096, 16, 101, 4
    X = pilots(dev, C - 1, seed=44)
    iq = ofdm.synth_frames(F, S, R, C, X, seed=45, noise_std=0.01)
    ws = ofdm.workspace(F, S, R, C, dev)
    ofdm.frame_estimate(iq, X, 0, ws)
    ref = ofdm.frame_combine(iq, 0, ws, ofdm.c64((F, S - 1, C - 1), dev))
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[ofdm.c64((F, S - 1, C - 1), dev) for _ in range(2)] for _ in range(4)]
    for o in outs:
        for t in o:
            t.fill_(float("nan"))
    torch.cuda.synchronize()
    for rep in range(4):
        for i in (0, 1):
            ofdm.frame_combine(iq, 0, ws, outs[rep][i], stream=sts[i])
    torch.cuda.synchronize()
    try:
        ofdm.device_status()
        reported = False
    except ofdm.OfdmError as e:
        assert "work-ticket" in str(e)
        reported = True
    bad = [(rep, i) for rep in range(4) for i in (0, 1) if not torch.equal(outs[rep][i], ref)]
    assert not bad or reported, bad
