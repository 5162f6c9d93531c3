"""Antenna-split orchestration (gpu-accel-ofdm-ls-mrc_amd/antenna_split.py) over
gloo, world_size 2, 3 and 8 (configs[4]: 256 antennas, 32 per rank), on CPU.

The collectives (all_reduce of |H|^2, reduce_scatter of the numerators, the
optional gather) are the real torch.distributed calls; the three kernel calls
are replaced by a numpy stand-in with the HIP library's signatures (NumpyOps
below, test-only).  The gathered result must match the oracle run on ALL
antennas within helpers.RTOL, and the ranks' finalised
slices must tile the output exactly once."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

from helpers import parity


def _out_pos(j, K):
    h = (K - 1) // 2
    return np.where(j >= h, j - h, j + (K + 1) // 2)


class NumpyOps:
    """CPU stand-in for ofdm_frame_ls_partial / ofdm_frame_mrc_partial /
    ofdm_mrc_finalize (same arguments and results; float64 FFT)."""

    @staticmethod
    def ls_partial(shard, X, prefix, ws=None, P=None, stream=None):
        import torch
        iq = shard.numpy()[:, 0, :, prefix:].astype(np.complex128)
        Y = np.fft.fft(iq, axis=-1)[..., 1:]
        Hc = np.conj(Y / X.numpy().astype(np.complex128)[None, None, :])
        p = (np.abs(Hc) ** 2).sum(axis=1).astype(np.float32)
        if P is None:
            P = torch.from_numpy(p)
        else:
            P.copy_(torch.from_numpy(p))
        return P, Hc

    @staticmethod
    def mrc_partial(shard, Hc, prefix, num=None, stream=None):
        import torch
        iq = shard.numpy()[:, 1:, :, prefix:].astype(np.complex128)
        Y = np.fft.fft(iq, axis=-1)[..., 1:]
        N = torch.from_numpy((Y * Hc[:, None]).sum(axis=2).astype(np.complex64))
        if num is None:
            return N
        num.copy_(N)
        return num

    @staticmethod
    def mrc_partial_range(shard, Hc, prefix, f0, count, num=None, stream=None):
        return NumpyOps.mrc_partial(shard[f0:f0 + count], Hc[f0:f0 + count], prefix, num=num, stream=stream)

    @staticmethod
    def mrc_finalize(chunk, e0, nsym, K, P, out, stream=None):
        c = chunk.numpy()
        e = e0 + np.arange(c.size)
        f, s, j = e // (nsym * K), (e // K) % nsym, e % K
        p = P.numpy()[f, j]
        o = out.numpy()  # shares memory with the torch tensor
        o[f, s, _out_pos(j, K)] = (c.real / p + 1j * (c.imag / p)).astype(np.complex64)
        return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, tmp, splits, prefix, gather, chunk=0):
    import torch
    import torch.distributed as dist
    import antenna_split
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(tmp, "in.npz"))
        r0, r1 = splits[rank], splits[rank + 1]
        shard = torch.from_numpy(np.ascontiguousarray(z["iq"][:, :, r0:r1]))
        X = torch.from_numpy(z["X"])
        if chunk:
            F, S = shard.shape[:2]
            K = shard.shape[-1] - prefix - 1
            pipe = antenna_split.SplitPipeline(F, S, r1 - r0, K + 1, prefix, "cpu",
                                               chunk_frames=chunk, ops=NumpyOps)
            out = torch.zeros((F, S - 1, K), dtype=torch.complex64)
            for _ in range(2):  # buffers reused across steps
                out.zero_()
                pipe.run(shard, X, out)
            # bench.py --mode split's stages_ms: one more step (rewrites the
            # same slices) and the collectives alone
            stages = pipe.profile_step(shard, X, out)
            with open(os.path.join(tmp, f"stages{rank}.json"), "w") as fp:
                json.dump(stages, fp)
            if gather:
                dist.all_reduce(torch.view_as_real(out))
            e0, count = 0, int((out != 0).sum())
        else:
            out, (e0, count) = antenna_split.demod_antenna_split(shard, X, prefix, ops=NumpyOps,
                                                                 gather=gather)
        np.savez(os.path.join(tmp, f"out{rank}.npz"), out=out.numpy(), e0=e0, count=count)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,R,F,S,C,prefix,gather,chunk", [
    (2, 8, 2, 4, 64, 0, True, 0),
    (2, 5, 3, 3, 256, 4, False, 0),    # uneven antenna split 3/2, CP dropped
    (3, 6, 1, 5, 16, 0, False, 0),     # element count not divisible by world
    (2, 8, 5, 4, 64, 0, True, 2),      # SplitPipeline: chunks 2+2+1 (short last chunk)
    (3, 7, 4, 3, 32, 2, False, 3),     # SplitPipeline: uneven split, padded chunks
    # configs[4]'s split: 256 antennas, 32 per rank, over 8 ranks
    (8, 256, 2, 3, 64, 0, True, 0),
    (8, 256, 3, 3, 64, 0, False, 0),
    (8, 256, 3, 3, 64, 0, True, 2),    # SplitPipeline: chunks 2+1
    (8, 256, 1, 3, 4096, 0, True, 1),  # configs[4]'s C
])
def test_antenna_split_gloo(oracle, world, R, F, S, C, prefix, gather, chunk):
    import torch.multiprocessing as mp
    rng = np.random.default_rng(world * 100 + R)
    K = C - 1
    iq = (rng.standard_normal((F, S, R, C + prefix)) +
          1j * rng.standard_normal((F, S, R, C + prefix))).astype(np.complex64)
    a = np.float32(0.70710678)
    X = (rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)
    splits = [round(i * R / world) for i in range(world + 1)]
    ref = oracle.frames_demod(iq, X, prefix)
    with tempfile.TemporaryDirectory() as tmp:
        np.savez(os.path.join(tmp, "in.npz"), iq=iq, X=X)
        mp.spawn(_worker, args=(world, _free_port(), tmp, splits, prefix, gather, chunk),
                 nprocs=world)
        res = [np.load(os.path.join(tmp, f"out{r}.npz")) for r in range(world)]
        if chunk:
            for r in range(world):
                with open(os.path.join(tmp, f"stages{r}.json")) as fp:
                    st = json.load(fp)
                for k in ("step_wall_ms", "all_reduce_alone_per_chunk", "reduce_scatter_alone_per_chunk",
                          "collectives_alone_step", "chunks"):
                    assert k in st and st[k] >= 0, (k, st)
                assert st["chunks"] == -(-F // chunk)
    n = F * (S - 1) * K
    if not (chunk and gather):
        assert sum(int(r["count"]) for r in res) == n
    assert [int(r["e0"]) for r in res] == sorted(int(r["e0"]) for r in res)
    if gather:
        for r in res:
            parity(r["out"], ref)
    else:
        # each output position is finalised by exactly one rank
        written = sum((r["out"] != 0).astype(int) for r in res)
        assert written.max() == 1 and written.sum() == n
        parity(sum(r["out"] for r in res), ref)


def test_slice_bounds():
    import antenna_split
    for n, world in [(10, 3), (9, 3), (0, 2), (5, 8)]:
        spans = [antenna_split.slice_bounds(n, world, r) for r in range(world)]
        assert sum(c for _, _, c in spans) == n
        pos = 0
        for _, e0, c in spans:
            if c:
                assert e0 == pos
            pos += c
