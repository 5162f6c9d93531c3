"""Antenna-split path through RCCL on the GPU (one rank: the box has one GPU;
the multi-rank orchestration is covered over gloo in test_antenna_split_cpu.py).
The result must equal frame_demod on all antennas within helpers.RTOL."""
import os
import socket

import numpy as np
import pytest

from helpers import parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.mark.parametrize("F,S,R,C,prefix", [(3, 6, 16, 1024, 0), (2, 4, 32, 4096, 0), (2, 5, 8, 256, 8)])
def test_antenna_split_rccl_matches_full(ofdm, dev, nccl_group, F, S, R, C, prefix):
    import torch
    import antenna_split
    rng = np.random.default_rng(C + R)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=21, noise_std=0.02)
    ref = ofdm.frame_demod(iq, X, prefix)
    out, (e0, count) = antenna_split.demod_antenna_split(iq, X, prefix, group=nccl_group, gather=True)
    torch.cuda.synchronize()
    assert (e0, count) == (0, F * (S - 1) * (C - 1))
    parity(out.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("F,S,R,C,prefix,chunk", [(5, 4, 32, 4096, 0, 2), (3, 6, 16, 1024, 8, 3)])
def test_split_pipeline_rccl_matches_full(ofdm, dev, nccl_group, F, S, R, C, prefix, chunk):
    """The chunked, overlapped pipeline bench.py --mode split times."""
    import torch
    import antenna_split
    rng = np.random.default_rng(C + R + 1)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=23, noise_std=0.02)
    ref = ofdm.frame_demod(iq, X, prefix)
    pipe = antenna_split.SplitPipeline(F, S, R, C, prefix, dev, group=nccl_group, chunk_frames=chunk)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    for _ in range(2):
        out.zero_()
        pipe.run(iq, X, out)
    torch.cuda.synchronize()
    parity(out.cpu().numpy(), ref.cpu().numpy())
