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
    def mrc_partial_range(shard, ws, prefix, f0, count, num=None, stream=None):
        import ofdm_lsmrc
        sd, wsd = HipOpsViaHost._ws
        N = ofdm_lsmrc.frame_mrc_partial_range(sd, wsd, prefix, f0, count).cpu()
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


def test_eight_shards_c4096_one_gpu_vs_oracle(ofdm, oracle, dev):
    """configs[4]'s split emulated on one GPU: 256 antennas as 8 shards of 32
    at C = 4096.  Each shard runs the HIP partial kernels
    (ofdm_frame_ls_partial / ofdm_frame_mrc_partial); the partial |H|^2 and
    numerators are summed over the shards in rank order (what all_reduce and
    reduce_scatter compute) and finalised by ofdm_mrc_finalize.  Reference:
    the oracle on all 256 antennas (findDistSqrd / matrixMultThenSum over
    every antenna, cpuLS.hpp:187-228)."""
    import torch
    F, S, G, Rg, C = 2, 4, 8, 32, 4096
    K = C - 1
    rng = np.random.default_rng(256)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K)).astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, G * Rg, C, X, seed=41, noise_std=0.02)
    P = torch.zeros((F, K), dtype=torch.float32, device=dev)
    num = torch.zeros((F, S - 1, K), dtype=torch.complex64, device=dev)
    for g in range(G):
        shard = iq[:, :, g * Rg:(g + 1) * Rg].contiguous()
        Pg, ws = ofdm.frame_ls_partial(shard, X)
        P += Pg
        num += ofdm.frame_mrc_partial(shard, ws)
    out = ofdm.c64((F, S - 1, K), dev)
    ofdm.mrc_finalize(num.reshape(-1), 0, S - 1, K, P, out)
    torch.cuda.synchronize()
    ref = oracle.frames_demod(iq.cpu().numpy(), X.cpu().numpy(), 0, nthreads=8)
    parity(out.cpu().numpy(), ref)
    assert int(ofdm.count_symbol_errors(out, S, seed=41).item()) == 0


def _bench(args, share, timeout=300):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "OFDM_BENCH_SHARE_GPU", "OFDM_BENCH_BACKEND"):
        env.pop(k, None)
    if share:
        env.update(OFDM_BENCH_SHARE_GPU="1", OFDM_BENCH_BACKEND="gloo")
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=root)


def _line(r):
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return __import__("json").loads(lines[0])


@pytest.mark.timeout(400)
def test_bench_gpus2_launches_two_ranks_itself():
    """`python bench.py --gpus 2` with no torchrun starts its two ranks
    itself (here sharing cuda:0 over gloo): n_gpus = 2, both ranks' frames
    counted, the timed output identical to the warm-up's."""
    line = _line(_bench(["--gpus", "2", "--frames", "24", "--steps", "2", "--warmup", "1", "--no-cpu"], True))
    assert line["n_gpus"] == 2 and line["config"]["global_data_symbols"] == 2 * 24 * 100
    assert line["check"]["qpsk_symbol_errors"] == 0 and line["check"]["timed_equals_warmup"] is True
    # per-rank spread of the step and kernel times
    pr = line["per_rank"]
    for k in ("step_ms", "kernel_ms"):
        assert 0 < pr[k]["min"] <= pr[k]["max"], pr


@pytest.mark.timeout(400)
def test_bench_split_rccl_world1_stage_times():
    """bench.py --mode split on RCCL (world 1, the product collective path):
    the line carries stages_ms -- the partial LS / FFT+MRC / finalise times,
    the communication left exposed by the overlap, and the collectives timed
    alone -- and the exposed time is within the step."""
    line = _line(_bench(["--mode", "split", "--frames", "8", "--chunk", "2", "--steps", "2", "--warmup", "1",
                         "--no-cpu"], False))
    st = line["stages_ms"]
    assert st["collective_path"] == "device (RCCL)"
    for k in ("ls_partial", "mrc_partial", "exposed_comm", "finalize", "step_events_ms", "all_reduce_alone_per_chunk",
              "reduce_scatter_alone_per_chunk", "collectives_alone_step"):
        assert k in st and st[k] >= 0, (k, st)
    assert st["exposed_comm"] <= st["step_events_ms"], st
    assert line["check"]["qpsk_symbol_errors"] == 0


@pytest.mark.timeout(200)
def test_bench_gpus2_refuses_on_one_gpu():
    """Asked for more GPUs than are visible, bench.py exits non-zero instead
    of measuring fewer."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    r = _bench(["--gpus", "2", "--frames", "8", "--steps", "1", "--warmup", "1", "--no-cpu"], False)
    assert r.returncode != 0 and not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "refusing" in r.stderr


@pytest.mark.timeout(600)
def test_bench_split_eight_ranks_share_gpu():
    """bench.py --mode split at configs[4]'s split (8 ranks x 32 antennas =
    256, C = 4096), the 8 ranks sharing cuda:0 over gloo: the gathered output
    of the timed steps matches the single-GPU receiver on all 256 antennas
    (check.vs_full_receiver, 1e-5)."""
    line = _line(_bench(["--mode", "split", "--gpus", "8", "--frames", "4", "--S", "5", "--chunk", "2",
                         "--steps", "1", "--warmup", "1", "--no-cpu"], True, timeout=560))
    assert line["n_gpus"] == 8 and line["config"]["R_total"] == 256 and line["config"]["C"] == 4096
    chk = line["check"]
    assert chk["qpsk_symbol_errors"] == 0 and chk["vs_full_receiver"]["ok"], chk


@pytest.mark.parametrize("C,F,S,R,prefix", [(4096, 9, 11, 4, 0), (1024, 7, 13, 3, 8), (2048, 6, 9, 2, 0),
                                            (1536, 5, 7, 2, 0)])
def test_mrc_partial_range_matches_chunk_workspaces(ofdm, dev, C, F, S, R, prefix):
    """ofdm_frame_mrc_partial_range (the pipelined split's MRC over one batch
    estimate) against ofdm_frame_ls_partial + ofdm_frame_mrc_partial on each
    chunk alone: the same kernels on the same frames, so bit-identical; a
    range outside the batch is refused."""
    import torch
    rng = np.random.default_rng(C + F)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1))
                         .astype(np.complex64)).to(dev)
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=C + 3, noise_std=0.02)
    _, ws = ofdm.frame_ls_partial(iq, X, prefix)
    for f0, cnt in ((0, 2), (2, 3), (5, F - 5), (0, F)):
        got = ofdm.frame_mrc_partial_range(iq, ws, prefix, f0, cnt)
        part = iq[f0:f0 + cnt].contiguous()
        _, wsc = ofdm.frame_ls_partial(part, X, prefix)
        ref = ofdm.frame_mrc_partial(part, wsc, prefix)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (f0, cnt)
    with pytest.raises(ofdm.OfdmError, match="outside"):
        ofdm.frame_mrc_partial_range(iq, ws, prefix, F - 1, 2)
