"""Streaming ingest (ofdm_pipeline_*) on the GPU:
host-resident frames -> pipelined H2D / fused receiver / D2H -> host outputs
must match the one-shot device path and the golden fixtures within
helpers.RTOL (not bit for bit: a chunk boundary changes which MRC workgroups
straddle two frames, and those take the per-wave Hc path of
k_mrc_td1024_hlds, whose FMA contraction differs in the last ulp); pageable and page-locked host
buffers, device buffers, chunk sizes that do not divide the batch, depth 1..4,
and the manual acquire/submit form the ring reader uses."""
import numpy as np
import pytest

from helpers import GOLDEN, parity

pytestmark = pytest.mark.gpu


def _golden(name):
    import os
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", ["r16_c1024_s4_2frames", "r4_c256_s5_cp32", "r8_c2048_s3_cp16",
                                  "r3_c64_s4_odd_antennas"])
def test_pipeline_golden(ofdm, dev, name):
    z = _golden(name)
    iq = np.ascontiguousarray(z["iq"], np.complex64)
    F, S, R, Cp = iq.shape
    prefix = int(z["prefix"])
    out = np.zeros((F, S - 1, Cp - prefix - 1), np.complex64)
    with ofdm.Pipeline(S, R, Cp - prefix, z["X"], prefix, chunk_frames=1, depth=2) as p:
        p.demod(iq, out)
        p.sync()
    parity(out, z["out"])


@pytest.mark.parametrize("F,chunk,depth,pinned", [(13, 4, 3, True), (13, 4, 3, False),
                                                  (7, 7, 1, True), (9, 2, 4, True),
                                                  (5, 8, 2, False)])
def test_pipeline_matches_device_path(ofdm, dev, F, chunk, depth, pinned):
    import torch
    S, R, C, prefix = 6, 64, 1024, 8
    rng = np.random.default_rng(F * 100 + chunk)
    a = np.float32(0.70710678)
    Xh = (rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)
    X = torch.from_numpy(Xh).to(dev)
    iq_d = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=F, noise_std=0.02)
    ref = ofdm.frame_demod(iq_d, X, prefix).cpu().numpy()
    iq = iq_d.cpu().numpy()
    out = np.zeros((F, S - 1, C - 1), np.complex64)
    if pinned:
        ofdm.host_register(iq)
        ofdm.host_register(out)
    try:
        with ofdm.Pipeline(S, R, C, Xh, prefix, chunk_frames=chunk, depth=depth) as p:
            p.demod(iq, out)
            p.sync()
            parity(out, ref)
            # second pass over the same pipeline (slots reused, events already recorded)
            out2 = np.zeros_like(out)
            if pinned:
                ofdm.host_register(out2)
            p.demod(iq, out2)
            p.sync()
            if pinned:
                ofdm.host_unregister(out2)
            assert np.array_equal(out2, out)  # same chunking: bit for bit
    finally:
        if pinned:
            ofdm.host_unregister(iq)
            ofdm.host_unregister(out)
    errs = int(ofdm.count_symbol_errors(torch.from_numpy(out).to(dev), S, seed=F).item())
    assert errs == 0


def test_pipeline_device_buffers_and_manual_slots(ofdm, dev):
    """Device input/output (hipMemcpyDefault) and the acquire / copy / submit
    sequence of the ring reader, with submit(n < chunk) and submit(0)."""
    import torch
    S, R, C, prefix, F = 5, 16, 2048, 16, 6
    rng = np.random.default_rng(3)
    Xh = (np.sign(rng.standard_normal(C - 1)) + 1j * np.sign(rng.standard_normal(C - 1))
          ).astype(np.complex64) * np.float32(0.70710678)
    X = torch.from_numpy(Xh).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=11, noise_std=0.01)
    ref = ofdm.frame_demod(iq, X, prefix)
    out = torch.zeros_like(ref)
    with ofdm.Pipeline(S, R, C, X, prefix, chunk_frames=4, depth=2) as p:
        p.demod(iq, out)
        p.sync()
        torch.cuda.synchronize()
        parity(out.cpu().numpy(), ref.cpu().numpy())
        # manual: frames 0..2 into one slot, nothing in the next, frames 3..5 in a third
        out.zero_()
        frame_bytes = iq[0].numel() * 8
        for lo, hi in ((0, 3), (3, 3), (3, 6)):
            d, s = p.acquire()
            n = hi - lo
            if n:
                _copy_to_ptr(d, iq[lo:hi], frame_bytes * n, s)
            p.submit(n, out[lo:hi] if n else None)
        p.sync()
        torch.cuda.synchronize()
        parity(out.cpu().numpy(), ref.cpu().numpy())


def _copy_to_ptr(dst_ptr, src, nbytes, stream):
    """Device-to-device copy of a contiguous tensor into a raw device pointer
    on the raw stream handle `stream` (hipMemcpyAsync of the HIP runtime
    torch has already loaded; kind 4 = hipMemcpyDefault)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpyAsync.restype = ctypes.c_int
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src.data_ptr()), nbytes, 4,
                            ctypes.c_void_p(stream))
    assert rc == 0, rc


def test_pipeline_rejects_bad_use(ofdm, dev):
    S, R, C = 3, 4, 256
    Xh = np.ones(C - 1, np.complex64)
    with ofdm.Pipeline(S, R, C, Xh, 0, chunk_frames=2, depth=2) as p:
        with pytest.raises(ofdm.OfdmError, match="no acquired slot"):
            p.submit(1)
        p.acquire()
        with pytest.raises(ofdm.OfdmError, match="already acquired"):
            p.acquire()
        with pytest.raises(ofdm.OfdmError, match="nframes out of"):
            p.submit(3)
        p.submit(0)
        p.sync()


def test_pipeline_ticketed_chunks_with_short_tail(ofdm, dev):
    """Chunks large enough for the one-launch demod's work tickets (48 frames
    x 100 symbols = 600 blocks) and a short last chunk (34 frames): a slot's
    workspace then serves two batch sizes, whose ticket counters sit at
    different offsets; two passes over the same pipeline, bit-identical, and
    within rounding of the one-shot device path."""
    import torch
    F, S, R, C, prefix = 130, 101, 2, 1024, 0
    rng = np.random.default_rng(130)
    a = np.float32(0.70710678)
    Xh = (rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)
    X = torch.from_numpy(Xh).to(dev)
    iq_d = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=130, noise_std=0.02)
    ref = ofdm.frame_demod(iq_d, X, prefix).cpu().numpy()
    iq = iq_d.cpu().numpy()
    with ofdm.Pipeline(S, R, C, Xh, prefix, chunk_frames=48, depth=2) as p:
        outs = []
        for _ in range(2):
            out = np.full((F, S - 1, C - 1), np.nan, np.complex64)
            p.demod(iq, out)
            p.sync()
            outs.append(out)
    parity(outs[0], ref)
    assert np.array_equal(outs[0], outs[1])
