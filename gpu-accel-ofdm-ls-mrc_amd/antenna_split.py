"""Antenna-split LS + MRC across ranks (BASELINE.json configs[4]).

Each rank holds every frame/symbol/subcarrier of ITS antennas (R_g of R; for
cfg5 256 antennas, 32 per GPU).  MRC is a sum over antennas, so

  P[f][j]    = sum_g P_g[f][j]        (partial |H|^2, findDistSqrd gpuLS.cu:185-209)
  N[f][s][j] = sum_g N_g[f][s][j]     (partial numerators, matrixMultThenSum
                                       cpuLS.hpp:187-208)
  out        = rotate(N / P)          (cpuLS.hpp:364-368, shiftOneRow 135-149)

Data path per batch (one process per GPU, RCCL over xGMI; SplitPipeline
runs step 1 once per batch and steps 3-5 in chunks):
  1. ofdm_frame_ls_partial     -> P_g, Hc_g (workspace)          local
  2. all_reduce(P)             F*K*4 B                           tiny
  3. ofdm_frame_mrc_partial    -> N_g (F*(S-1)*K complex)        local, HBM-bound
  4. reduce_scatter(N)         each rank receives 1/world of the flattened
                               numerators, summed: the per-link traffic of a
                               ring reduce-scatter is (world-1)/world * |N|/world
                               per step, spread over the xGMI links, vs a full
                               all-reduce's 2x
  5. ofdm_mrc_finalize         divide + rotate of the rank's slice into `out`
                               (elements of that slice only; other positions
                               are left untouched)
  optional 6. all_reduce(out)  (zeros elsewhere) when every rank needs all of it

The kernel calls go through `ops` (default: the HIP library, ofdm_lsmrc).  A
CPU stand-in with the same signatures is used by tests/test_antenna_split_cpu.py
to check this orchestration over gloo; the product path has no CPU fallback.
"""
import ofdm_lsmrc


class HipOps:
    """The HIP library calls used by the antenna-split path."""
    ls_partial = staticmethod(ofdm_lsmrc.frame_ls_partial)        # (shard, X, prefix) -> (P, ws)
    mrc_partial = staticmethod(ofdm_lsmrc.frame_mrc_partial)      # (shard, ws, prefix) -> N
    mrc_partial_range = staticmethod(ofdm_lsmrc.frame_mrc_partial_range)  # (shard, ws, prefix, f0, count) -> N
    mrc_finalize = staticmethod(ofdm_lsmrc.mrc_finalize)          # (chunk, e0, nsym, K, P, out)


def slice_bounds(n, world, rank):
    """Flat element range [e0, e0 + count) that `rank` finalises when `n`
    numerators are reduce-scattered in equal chunks of ceil(n / world)."""
    per = -(-n // world) if n else 0
    e0 = min(rank * per, n)
    return per, e0, max(0, min(per, n - e0))


def demod_antenna_split(shard, X, prefix=0, group=None, ops=HipOps, gather=False, out=None):
    """LS + MRC of frames whose antennas are split across the ranks of `group`.

    shard: (F, S, R_g, C + prefix) complex64, this rank's antennas (any R_g >= 1;
           ranks may hold different counts).
    X:     (K,) rotated pilots (matrix_readX), identical on every rank.
    Returns (out, (e0, count)): out is (F, S-1, K) complex64 with this rank's
    finalised flat numerator range [e0, e0 + count) written at its rotated
    output positions (all positions when gather=True; a caller-supplied `out`
    must then be zero-filled, since the gather is a sum over ranks).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    F, S, _, Cp = shard.shape
    K = Cp - prefix - 1
    P, ws = ops.ls_partial(shard, X, prefix)
    dist.all_reduce(P, group=group)
    num = ops.mrc_partial(shard, ws, prefix)
    n = num.numel()
    per, e0, count = slice_bounds(n, world, rank)
    flat = torch.view_as_real(num).reshape(-1)
    if per * world != n:
        flat = torch.cat([flat, flat.new_zeros(2 * (per * world - n))])
    mine = flat.new_empty(2 * per)
    dist.reduce_scatter_tensor(mine, flat, group=group)
    if out is None:
        out = torch.zeros((F, S - 1, K), dtype=torch.complex64, device=shard.device)
    if count:
        chunk = torch.view_as_complex(mine[:2 * count].view(count, 2))
        ops.mrc_finalize(chunk, e0, S - 1, K, P, out)
    if gather:
        dist.all_reduce(torch.view_as_real(out), group=group)
    return out, (e0, count)


class SplitPipeline:
    """Chunked, overlapped antenna-split LS + MRC for a fixed batch shape
    (bench.py --mode split).

    One partial LS over the whole batch (one launch: a workgroup per frame
    fills the GPU, where per-chunk LS launches of `chunk_frames` workgroups
    left most CUs idle) -> async all_reduce(P) of every frame; then the MRC
    streams in chunks of `chunk_frames`, on the caller's stream: partial MRC
    of chunk c (ofdm_frame_mrc_partial_range on the batch's estimate) ->
    async reduce_scatter(numerators); the collectives of chunk c run on the
    RCCL stream while chunk c+1 computes, and chunk c is finalised (divide +
    rotate of this rank's slice) once both have landed.  Buffers are
    allocated once (the numerators double-buffered), so a step issues no
    allocation.  `ops` as for demod_antenna_split (the kernel calls take the
    preallocated ws / P / num and the stream as keyword arguments).
    Each rank writes only its slices of `out` (see demod_antenna_split).
    """

    def __init__(self, F, S, R_local, C, prefix, device, group=None, chunk_frames=50, ops=HipOps):
        import torch
        import torch.distributed as dist
        self.F, self.S, self.R, self.C, self.prefix = F, S, R_local, C, prefix
        self.K = C - 1
        self.group = group
        self.ops = ops
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.chunk = max(1, min(chunk_frames, F))
        fc = self.chunk
        n = fc * (S - 1) * self.K
        self.per = -(-n // self.world)
        self.ws = ofdm_lsmrc.workspace(F, S, R_local, C, device) if ops is HipOps else None
        self.P = torch.empty((F, self.K), dtype=torch.float32, device=device)
        # numerators padded to world * per complex values (padding stays 0)
        self.num = [torch.zeros(self.per * self.world, dtype=torch.complex64, device=device)
                    for _ in range(2)]
        self.mine = [torch.empty(self.per, dtype=torch.complex64, device=device) for _ in range(2)]
        # rehearsal of N ranks on fewer GPUs over gloo (bench.py with
        # OFDM_BENCH_BACKEND=gloo, tests): gloo's reduce-scatter takes host
        # tensors only, so both collectives go through host copies,
        # synchronously.  RCCL (the product backend) never takes this branch.
        self.host_coll = (dist.get_backend(group) == "gloo" and torch.device(device).type == "cuda")

    def run(self, shard, X, out, stream=None, timing=None):
        """shard: (F, S, R_local, C + prefix) on this rank; out: (F, S-1, K).
        stream: a torch.cuda.Stream to run on (default: the current stream).
        The whole step -- kernels, collectives and their waits -- is issued
        with `stream` as torch's current stream, because the async
        collectives and work.wait() order themselves against the current
        stream: kernels on any other stream could race them.
        timing: a dict to receive HIP events of the step's stages on that
        stream (profile_step; never in a timed step)."""
        if stream is not None and self.ops is HipOps:
            import torch
            with torch.cuda.stream(stream):
                return self._run(shard, X, out, timing=timing)
        return self._run(shard, X, out, timing=timing)

    def profile_step(self, shard, X, out, stream=None):
        """Stage times of ONE step (ms, HIP events on the compute stream), for
        a SCALE run that falls short: the partial LS, the partial FFT+MRC and
        the finalise summed over chunks; `exposed_comm` = the time the
        compute stream spent blocked in the waits for the collectives (what
        the overlap did not hide); and the two collectives timed alone
        (issued and waited one by one on the last chunk's buffers), so
        exposed can be read against what they cost."""
        import time
        import torch
        import torch.distributed as dist
        if stream is None:
            stream = torch.cuda.current_stream() if torch.cuda.is_available() and self.ops is HipOps else None
        ev = {}
        if stream is not None:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.run(shard, X, out, stream=stream, timing=ev)
        if stream is not None:
            torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3

        def span(a, b):
            return sum(x.elapsed_time(y) for x, y in zip(ev.get(a, []), ev.get(b, [])))
        st = {"step_wall_ms": wall}
        if ev:
            st.update({"ls_partial": span("ls0", "ls1"), "mrc_partial": span("m0", "mrc1"),
                       "exposed_comm": span("w0", "w1"), "finalize": span("w1", "fin1"),
                       "step_events_ms": ev["ls0"][0].elapsed_time(ev["fin1"][-1])})
        # the collectives alone, on the last buffers used
        b = 0
        fc = min(self.chunk, self.F)
        iso = {}  # (the all-reduce of one chunk's P, as the per-chunk form issued it)
        for name in ("all_reduce", "reduce_scatter"):
            if stream is not None:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name == "all_reduce":
                if self.host_coll:
                    Ph = self.P[:fc].cpu()
                    dist.all_reduce(Ph, group=self.group)
                else:
                    dist.all_reduce(self.P[:fc], group=self.group)
            else:
                if self.host_coll:
                    mine_h = torch_real(self.mine[b]).cpu()
                    dist.reduce_scatter_tensor(mine_h, torch_real(self.num[b]).cpu(), group=self.group)
                else:
                    dist.reduce_scatter_tensor(torch_real(self.mine[b]), torch_real(self.num[b]),
                                               group=self.group)
            if stream is not None:
                torch.cuda.synchronize()
            iso[name] = (time.perf_counter() - t0) * 1e3
        nchunks = -(-self.F // self.chunk)
        st.update({"all_reduce_alone_per_chunk": iso["all_reduce"],
                   "reduce_scatter_alone_per_chunk": iso["reduce_scatter"],
                   "chunks": nchunks,
                   "collectives_alone_step": iso["all_reduce"] + iso["reduce_scatter"] * nchunks,
                   "collective_path": "host-staged (gloo rehearsal)" if self.host_coll else "device (RCCL)"})
        return st

    def _run(self, shard, X, out, stream=None, timing=None):
        import torch
        import torch.distributed as dist
        F, S, K = self.F, self.S, self.K
        pending = []
        reduced = {"P": None}  # the async all-reduce of P, waited for once

        def mark(name):  # HIP events on the current stream (kernel stand-ins of the CPU tests: none)
            if timing is not None and self.ops is HipOps:
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                timing.setdefault(name, []).append(e)

        def finalize(c, b, wn):
            mark("w0")
            if reduced["P"] is not None:
                reduced["P"].wait()
                reduced["P"] = None
            if wn is not None:
                wn.wait()
            mark("w1")
            f0 = c * self.chunk
            fc = min(self.chunk, F - f0)
            n = fc * (S - 1) * K
            e0 = min(self.rank * self.per, n)
            count = max(0, min(self.per, n - e0))
            if count:
                self.ops.mrc_finalize(self.mine[b][:count], e0, S - 1, K, self.P[f0:f0 + fc],
                                      out[f0:f0 + fc], stream=stream)
            mark("fin1")

        mark("ls0")
        _, self.ws = self.ops.ls_partial(shard, X, self.prefix, ws=self.ws, P=self.P, stream=stream)
        mark("ls1")
        if self.host_coll:
            Ph = self.P.cpu()
            dist.all_reduce(Ph, group=self.group)
            self.P.copy_(Ph)
        else:
            reduced["P"] = dist.all_reduce(self.P, group=self.group, async_op=True)
        nchunks = -(-F // self.chunk)
        for c in range(nchunks):
            b = c & 1
            f0 = c * self.chunk
            fc = min(self.chunk, F - f0)
            n = fc * (S - 1) * K
            num = self.num[b][:n].view(fc, S - 1, K)
            mark("m0")
            self.ops.mrc_partial_range(shard, self.ws, self.prefix, f0, fc, num=num, stream=stream)
            mark("mrc1")
            flat = self.num[b] if n == self.per * self.world else self._padded(b, n)
            if self.host_coll:
                mine_h = torch_real(self.mine[b]).cpu()
                dist.reduce_scatter_tensor(mine_h, torch_real(flat).cpu(), group=self.group)
                torch_real(self.mine[b]).copy_(mine_h)
                wn = None
            else:
                wn = dist.reduce_scatter_tensor(torch_real(self.mine[b]), torch_real(flat),
                                                group=self.group, async_op=True)
            pending.append((c, b, wn))
            if len(pending) == 2:
                finalize(*pending.pop(0))
        while pending:
            finalize(*pending.pop(0))
        return out

    def _padded(self, b, n):
        # a short last chunk: zero the tail so stale numerators are not summed
        self.num[b][n:].zero_()
        return self.num[b]


def torch_real(t):
    import torch
    return torch.view_as_real(t).reshape(-1)
