"""Antenna-split path on the GPU.

* Through RCCL with one rank (the box has one GPU): the result must equal the
  oracle (the C restatement of cpuLS.hpp) on all antennas within
  helpers.RTOL.
* With two ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one
  GPU): the HIP partial kernels (ofdm_frame_ls_partial / _mrc_partial /
  ofdm_mrc_finalize) inside a real 2-rank job, each rank holding half of the
  antennas, the collectives on host copies of the kernels' outputs (gloo's
  reduce-scatter is host-only); gathered result vs the oracle on all antennas.
* The frame-sharded bench step (bench.py's N > 1 path: per-rank frame0,
  barrier + max-over-ranks timing, error sum) with two ranks on cuda:0."""
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
def test_antenna_split_rccl_vs_oracle(ofdm, oracle, dev, nccl_group, F, S, R, C, prefix):
    import torch
    import antenna_split
    rng = np.random.default_rng(C + R)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=21, noise_std=0.02)
    out, (e0, count) = antenna_split.demod_antenna_split(iq, X, prefix, group=nccl_group, gather=True)
    torch.cuda.synchronize()
    assert (e0, count) == (0, F * (S - 1) * (C - 1))
    parity(out.cpu().numpy(), oracle.frames_demod(iq.cpu().numpy(), X.cpu().numpy(), prefix, nthreads=8))


@pytest.mark.parametrize("F,S,R,C,prefix,chunk", [(5, 4, 32, 4096, 0, 2), (3, 6, 16, 1024, 8, 3)])
def test_split_pipeline_rccl_vs_oracle(ofdm, oracle, dev, nccl_group, F, S, R, C, prefix, chunk):
    """The chunked, overlapped pipeline bench.py --mode split times."""
    import torch
    import antenna_split
    rng = np.random.default_rng(C + R + 1)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=23, noise_std=0.02)
    ref = oracle.frames_demod(iq.cpu().numpy(), X.cpu().numpy(), prefix, nthreads=8)
    pipe = antenna_split.SplitPipeline(F, S, R, C, prefix, dev, group=nccl_group, chunk_frames=chunk)
    out = ofdm.c64((F, S - 1, C - 1), dev)
    st = torch.cuda.Stream(device=dev)  # a non-current stream: the whole step must follow it
    for _ in range(2):
        out.zero_()
        torch.cuda.synchronize()
        pipe.run(iq, X, out, stream=st)
        st.synchronize()
    parity(out.cpu().numpy(), ref)


class HipOpsViaHost:
    """The HIP library's antenna-split kernels on cuda:0, their inputs and
    outputs staged through host memory so that the orchestration and its gloo
    collectives run on CPU tensors (test-only adapter)."""

    @staticmethod
    def ls_partial(shard, X, prefix, ws=None, P=None, stream=None):
        import ofdm_lsmrc
        Pd, wsd = ofdm_lsmrc.frame_ls_partial(shard.cuda(), X.cuda(), prefix)
        HipOpsViaHost._ws = (shard.cuda(), wsd)
        if P is None:
            return Pd.cpu(), wsd
        P.copy_(Pd.cpu())
        return P, wsd

    @staticmethod
    def mrc_partial(shard, ws, prefix, num=None, stream=None):
        import ofdm_lsmrc
        sd, wsd = HipOpsViaHost._ws
        N = ofdm_lsmrc.frame_mrc_partial(sd, wsd, prefix).cpu()
        if num is None:
            return N
        num.copy_(N)
        return num

    @staticmethod
    def mrc_finalize(chunk, e0, nsym, K, P, out, stream=None):
        import ofdm_lsmrc
        od = out.cuda()
        ofdm_lsmrc.mrc_finalize(chunk.cuda(), e0, nsym, K, P.cuda(), od)
        out.copy_(od.cpu())
        return out


def _two_rank_worker(rank, world, port, tmp, splits, prefix, chunk):
    import torch
    import torch.distributed as dist
    import antenna_split
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(tmp, "in.npz"))
        r0, r1 = splits[rank], splits[rank + 1]
        shard = torch.from_numpy(np.ascontiguousarray(z["iq"][:, :, r0:r1]))
        X = torch.from_numpy(z["X"])
        F, S = shard.shape[:2]
        K = shard.shape[-1] - prefix - 1
        if chunk:
            pipe = antenna_split.SplitPipeline(F, S, r1 - r0, K + 1, prefix, "cpu", chunk_frames=chunk,
                                               ops=HipOpsViaHost)
            out = torch.zeros((F, S - 1, K), dtype=torch.complex64)
            pipe.run(shard, X, out)
            dist.all_reduce(torch.view_as_real(out))
        else:
            out, _ = antenna_split.demod_antenna_split(shard, X, prefix, ops=HipOpsViaHost, gather=True)
        np.save(os.path.join(tmp, f"out{rank}.npy"), out.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("F,S,R,C,prefix,chunk", [(3, 5, 16, 1024, 0, 0), (2, 3, 32, 4096, 4, 0),
                                                  (4, 4, 12, 2048, 0, 3)])
def test_antenna_split_two_ranks_hip_kernels_vs_oracle(ofdm, oracle, dev, tmp_path, F, S, R, C, prefix,
                                                       chunk):
    import torch
    import torch.multiprocessing as mp
    rng = np.random.default_rng(F * 10 + R)
    a = np.float32(0.70710678)
    K = C - 1
    Xh = (rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)
    iq = ofdm.synth_frames(F, S, R, C, torch.from_numpy(Xh).to(dev), prefix=prefix, seed=31,
                           noise_std=0.02).cpu().numpy()
    np.savez(tmp_path / "in.npz", iq=iq, X=Xh)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_two_rank_worker, args=(2, port, str(tmp_path), [0, R // 2, R], prefix, chunk), nprocs=2)
    ref = oracle.frames_demod(iq, Xh, prefix, nthreads=8)
    for r in range(2):
        parity(np.load(tmp_path / f"out{r}.npy"), ref)


def test_frame_sharded_bench_two_ranks(tmp_path):
    """bench.py's N = 2 path on one GPU (OFDM_BENCH_SHARE_GPU=1, gloo): every
    rank demodulates its own frame range with zero QPSK errors and rank 0
    prints one whole-job line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OFDM_BENCH_SHARE_GPU="1", OFDM_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--frames", "24", "--steps", "2", "--warmup", "1", "--no-cpu"],
                       capture_output=True, text=True, timeout=180, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_data_symbols"] == 2 * 24 * 100
    assert line["check"]["qpsk_symbol_errors"] == 0
