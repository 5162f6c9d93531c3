#!/usr/bin/env python3
"""Benchmark: OFDM LS + MRC receiver throughput on MI355X.

Workload (BASELINE.json metric "OFDM symbols/s (LS+MRC) at 1024 subcarriers x
64 ant"; configs[3] "8xMI355X: 1024 subcarriers, 64 antennas, 1M symbols
sharded by symbol index (no RCCL), per-GPU hipStreams"): each GPU holds
`--frames` frames (default 1250) of S = 101 symbols (1 pilot + 100 data,
lenOfBuffer of ShMemSymBuff_gpu.hpp:74) x R = 64 antennas x C = 1024
time-domain IQ samples, synthetic, resident in HBM (66 GB per GPU).  One step =
ofdm_frame_demod over the whole batch (pilot FFT + LS, FFT + MRC + normalise +
rotate): 125,000 data symbols per GPU, 1M at 8 GPUs (weak scaling,
frame-sharded, no collective on the data path).  At C = 1024 that is ONE
launch (k_demod_td1024: estimator and MRC workgroups in one grid); --flow two
runs and times ofdm_frame_estimate + ofdm_frame_combine separately.

value = data symbols demodulated per second, whole job (all ranks).
roofline: dominant kernel, algorithmic bytes per data symbol
  B_sym = R*C*8 (IQ read once) + K*8 (output written once), for the
  one-launch kernel + R*C*8 + K*8 per frame (pilot symbol, pilot vector),
  divided by its HIP-event-measured average launch time, vs 8 TB/s HBM3E.
cpu_baseline: the oracle's C restatement of cpuLS.hpp (oracle/) with its
  single-precision radix-2 FFT (the reference's fftwf precision; the parity
  oracle keeps a float64 FFT) timed on this host, rank 0 at N=1, on a bounded
  sample of frames of the same shape, OpenMP over frames.

python bench.py [--gpus N] [--steps K] [--warmup W]
torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

`python bench.py --gpus N` (N > 1) without torchrun starts the N ranks
itself: the launcher process never touches the GPU (it only counts the
visible devices, which does not initialise HIP), starts N fresh child
processes of this script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
and exits with their status.  Fewer visible GPUs than N is an error (exit
2), never a silent scale-down; OFDM_BENCH_SHARE_GPU=1 (tests only) maps the
ranks onto the visible GPUs round-robin.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["frames", "freq", "split", "pcie"], default="frames",
                    help="frames: frame-sharded receiver (configs[3], the headline); freq: the "
                         "same frames in the frequency domain (FFT upstream: LS + MRC alone, "
                         "SURVEY.md 8(d) mode A); split: "
                         "antenna-split partial MRC + RCCL (configs[4]), --R antennas per GPU; "
                         "pcie: host-resident frames through ofdm_pipeline (H2D + receiver + "
                         "D2H overlapped; PCIe-inclusive rate, never the headline)")
    ap.add_argument("--depth", type=int, default=3, help="pcie: pipeline slots")
    ap.add_argument("--frames", type=int, default=None, help="frames per GPU (1250; split: 400)")
    ap.add_argument("--S", type=int, default=101)
    ap.add_argument("--R", type=int, default=None, help="antennas per GPU (64; split: 32)")
    ap.add_argument("--C", type=int, default=None, help="subcarriers (1024; split: 4096)")
    ap.add_argument("--chunk", type=int, default=None,
                    help="frames per pipelined chunk (split: 50, pcie: 4)")
    ap.add_argument("--prefix", type=int, default=0)
    ap.add_argument("--flow", choices=["auto", "one", "two"], default="auto",
                    help="frames mode: 'one' = ofdm_frame_demod (LS and MRC in one launch, C = 1024), "
                         "'two' = ofdm_frame_estimate + ofdm_frame_combine timed separately; auto: one at "
                         "C = 1024 in the time domain, else two")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--noise", type=float, default=0.01)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-box", action="store_true",
                    help="skip the same-box HBM probes and the diagnostic-build clock reading")
    ap.add_argument("--stamps-out", default=None,
                    help="save the diagnostic build's per-workgroup stamps (.npy) for scripts/wg_timeline.py")
    ap.add_argument("--no-mode-a", action="store_true",
                    help="skip the supplementary frequency-domain (mode A) measurement of the default mode")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC traffic summary (profiles/) for roofline.traffic")
    args = ap.parse_args()
    split = args.mode == "split"
    args.chunk = args.chunk or (4 if args.mode == "pcie" else 50)
    args.frames = args.frames or (400 if split else 48 if args.mode == "pcie" else 1250)
    args.R = args.R or (32 if split else 64)
    args.C = args.C or (4096 if split else 1024)
    return args


def cpu_baseline(args, X, ofdm, torch, dev):
    """Oracle (C restatement of cpuLS.hpp) on the host cores of this box
    (--mode freq: its LS + MRC on frequency-domain frames, no FFT)."""
    freq = args.mode == "freq"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_bindings import Oracle
    o = Oracle()
    share = host_cpu_share()
    threads = share["threads"]
    Xh = X.cpu().numpy()

    def sample(nf):
        iq = ofdm.synth_frames(nf, args.S, args.R, args.C, X, prefix=args.prefix,
                               seed=args.seed + 7, noise_std=args.noise, freq_domain=freq)
        torch.cuda.synchronize()
        return iq.cpu().numpy()

    def run(iq):
        if freq:
            o.frames_demod_freq(iq, Xh, nthreads=threads)
        else:  # single-precision FFT, the precision class of the reference's fftwf, vectorised
            o.frames_demod_fast(iq, Xh, args.prefix, nthreads=threads)

    iq1 = sample(threads)
    t0 = time.perf_counter()
    run(iq1)
    t1 = time.perf_counter() - t0
    nf = max(threads, int(args.cpu_seconds / max(t1, 1e-3) * threads) // threads * threads)
    frame_bytes = args.S * args.R * (args.C + (0 if freq else args.prefix)) * 8
    nf = min(nf, 64 * threads, max(threads, int(16e9 // frame_bytes) // threads * threads))  # <= 16 GB host
    iq = sample(nf) if nf != threads else iq1
    passes, t0 = 0, time.perf_counter()
    while passes < 1 or time.perf_counter() - t0 < min(3.0, args.cpu_seconds):  # >= 3 s of host work
        run(iq)
        passes += 1
    dt = time.perf_counter() - t0
    syms = passes * nf * (args.S - 1)
    # BASELINE configs[0] / SURVEY.md 8(d)(a): the cpuLS.hpp shape (R=4, C=1024,
    # one frame of 100 symbols = 1 pilot + 99 data) on ONE host thread
    c1 = ofdm.synth_frames(1, 100, 4, 1024, X, prefix=0, seed=args.seed + 11, noise_std=args.noise)
    torch.cuda.synchronize()
    c1 = c1.cpu().numpy()
    reps, t0 = 0, time.perf_counter()
    while reps < 5 or time.perf_counter() - t0 < 1.0:
        o.frames_demod_fast(c1, Xh, 0, nthreads=1)
        reps += 1
    d1 = time.perf_counter() - t0
    fft = "none (frequency-domain input)" if freq else \
        "float32 radix-2, AVX2-vectorised (oracle/fft_fast.c: split arrays, unit-stride per-stage twiddles, AVX2 " \
        "code behind a runtime CPU check, no FMA contraction; bit-identical to the scalar oracle_fft_row_f32; " \
        "FFTW's codelets are not available here)"
    # cores = the threads the sample ran on (the bench contract), i.e. the
    # CPU share this job has on the box (cgroup quota, else the affinity
    # mask, else os.cpu_count()); how that share was read is reported beside it
    return {"value": syms / dt, "unit": "symbols/s", "cores": threads, "threads": threads,
            "cpu_share": share, "kind": "port", "fft": fft,
            "sample": f"{passes} x {nf} frames x {args.S} symbols (R={args.R}, C={args.C}, prefix="
                      f"{args.prefix}), {'LS+MRC+rotate (frequency domain)' if freq else 'FFT+LS+MRC+rotate'}, "
                      f"FFT: {'none' if freq else 'float32 radix-2, vectorised'}, OpenMP over frames, "
                      f"{dt:.1f} s wall", "seconds": dt,
            "configs0_single_thread": {"value": reps * 99 / d1, "unit": "symbols/s", "cores": 1, "fft": fft,
                                       "sample": f"R=4, C=1024, 1 frame x 100 symbols, {reps} repetitions, "
                                                 f"FFT float32 radix-2 vectorised, {d1:.2f} s wall"}}


def host_cpu_share():
    """The CPU share of this job, read from the box: the cgroup v2 quota
    (cpu.max "quota period", or v1 cfs_quota_us / cfs_period_us), else the
    affinity mask, else os.cpu_count().  threads = the share rounded down
    (at least 1), capped by the affinity mask."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota, src = None, None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as fp:
                q, per = fp.read().split()[:2]
            if q != "max":
                quota, src = int(q) / int(per), path
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fp:
                q = int(fp.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fp:
                per = int(fp.read())
            if q > 0:
                quota, src = q / per, "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
        except (OSError, ValueError):
            pass
    if quota is not None:
        threads = max(1, min(affinity, int(quota)))
    else:
        threads, src = affinity, "sched_getaffinity"
    return {"threads": threads, "cgroup_quota_cpus": quota, "affinity_cpus": affinity,
            "os_cpu_count": os.cpu_count(), "source": src}


def box_probe(ofdm, torch, dev, stream, gib=4, reps=5):
    """Same-box HBM ceilings, timed in this process right after the timed
    loop: a float4 copy of `gib` GiB (read + written bytes counted) and a
    float4 read of the same source (ofdm_hbm_probe, plain 16-B accesses over
    the whole chip).  Median of `reps` launches by HIP events."""
    n = gib << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev)
    src.view(torch.float32).uniform_()
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    res = {}
    for mode, name, moved in ((0, "copy", 2 * n), (1, "read", n)):
        sink = dst if mode == 0 else dst[: 8 << 20]
        ofdm.hbm_probe(mode, src, sink, stream)  # warm
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ofdm.hbm_probe(mode, src, sink, stream)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[name] = moved / (ts[len(ts) // 2] * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return {"box_copy_GBps": res["copy"], "box_read_GBps": res["read"],
            "box_probe": f"ofdm_hbm_probe over {gib} GiB (16 KiB non-temporal chunks per wave, 16 loads per lane in flight), median of {reps}; copy counts read + written bytes"}


DIAG_LIB = os.path.join(ROOT, "gpu-accel-ofdm-ls-mrc_amd", "lib", "libofdm_lsmrc_diag.so")
DIAG_TAG = {1024: "td1024", 2048: "td2048", 4096: "td4096"}


def stamps_summary(rec):
    """Per-workgroup records of the diagnostic build (csrc/diag.hpp): rt0,
    rt_mark, rt_end (100 MHz), mt0, mt_end (shader clock), hw_id, xcc_id,
    block.  Effective clock = d(memtime) / d(memrealtime) x 100 MHz."""
    import numpy as np
    rec = rec[rec[:, 2] > 0]
    if not len(rec):
        return None
    drt = (rec[:, 2] - rec[:, 0]).astype(np.float64)
    dmt = (rec[:, 4] - rec[:, 3]).astype(np.float64)
    ok = drt > 0
    ghz = dmt[ok] / drt[ok] * 0.1
    span = (rec[:, 2].max() - rec[:, 0].min()) * 1e-5  # ms
    return {"effective_GHz_median": float(np.median(ghz)), "effective_GHz_p10": float(np.percentile(ghz, 10)),
            "effective_GHz_p90": float(np.percentile(ghz, 90)),
            "busy_weighted_GHz": float(dmt[ok].sum() / drt[ok].sum() * 0.1),
            "workgroups": int(len(rec)), "stamped_span_ms": float(span)}


def clock_probe(step_diag, tag, ofdm, torch, stream, reps=3, save=None):
    """Effective clock of the timed kernel: the diagnostic build of the SAME
    kernel (make diag; per-workgroup s_memtime / s_memrealtime stamps, no
    other change) run `reps` times right after the timed loop on the same
    batch; the stamps of the last launch give the clock per workgroup."""
    import ctypes
    import numpy as np
    if not os.path.exists(DIAG_LIB) or tag is None:
        return None
    L = ofdm.load_library(DIAG_LIB)
    clear, read = getattr(L, f"ofdm_diag_clear_{tag}"), getattr(L, f"ofdm_diag_read_{tag}")
    read.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    ts = []
    with ofdm.using(L):
        for i in range(reps):
            torch.cuda.synchronize()
            if i == reps - 1:
                clear()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            step_diag()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
    nwg = 1 << 20  # diag::MAX_WG (the last launch's records may sit in any slot; the buffer was cleared before it)
    rec = np.zeros((nwg, 12), dtype=np.uint64)  # diag::WORDS
    if read(rec.ctypes.data, nwg) != 0:
        return None
    if save:
        np.save(save, rec[rec[:, 2] > 0])
    out = stamps_summary(rec)
    if out is None:
        return None
    out.update({"diag_launch_ms": ts, "source": f"lib/libofdm_lsmrc_diag.so (the same kernel with per-workgroup "
                                                f"s_memtime/s_memrealtime stamps, csrc/diag.hpp), {reps} launches "
                                                f"right after the timed loop, stamps of the last"})
    return out


def pmc_traffic(path, cfg, build):
    """Corrected PMC HBM bytes per launch for this exact config AND this
    build of the library (`build`: ofdm_lsmrc.build_id(), which
    scripts/pmc_summary.py records from the profiled run's bench line): `path`
    (profiles/pmc_traffic.json, the default shape) or else the latest-tagged
    profiles/r*_traffic.json for it.  A profile of other code is never
    credited: (None, "no profile of this build")."""
    cands = [path] + sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")) +
                            glob.glob(os.path.join(ROOT, "profiles", "r*", "r*_traffic.json")),
                            key=os.path.basename, reverse=True)
    for p in cands:
        try:
            with open(p) as fp:
                d = json.load(fp)
        except (OSError, ValueError):
            continue
        dc = d.get("config", {})
        if all(dc.get(k) == cfg[k] for k in ("R", "C", "S", "frames_per_gpu", "prefix")) and \
                dc.get("domain", "time") == cfg["domain"] and \
                dc.get("flow", "two-launch") == cfg.get("flow", "two-launch") and \
                d.get("build_id") == build:
            return d.get("mrc_hbm_bytes_per_launch"), os.path.relpath(p, ROOT)
    return None, "no profile of this build"


def visible_gpus():
    """Visible device count without initialising HIP in this process
    (torch.cuda.device_count() does not, on this image)."""
    import torch
    return torch.cuda.device_count()


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """--gpus N > 1 without a launcher: N fresh child processes of this
    script, one per GPU (never an exec of this process).  Returns the exit
    status: the first non-zero child status (the others are then
    terminated, so no rank waits forever in a collective), else 0."""
    share = os.environ.get("OFDM_BENCH_SHARE_GPU") == "1"
    have = visible_gpus()
    if have < n and not share:
        log(f"error: --gpus {n} but only {have} GPU(s) visible; refusing to run fewer ranks "
            f"(OFDM_BENCH_SHARE_GPU=1 shares GPUs for rehearsals only)")
        return 2
    if have < 1:
        log("error: no GPU visible")
        return 2
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            st = p.poll()
            if st is None:
                continue
            live.remove(p)
            if st != 0 and rc == 0:
                rc = st if st > 0 else 1
                log(f"error: rank {procs.index(p)} exited with status {st}; stopping the other ranks")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist
    import ofdm_lsmrc as ofdm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    # rehearsal of the N > 1 path on fewer GPUs (tests only, never the
    # measurement): OFDM_BENCH_SHARE_GPU=1 maps ranks onto the visible GPUs
    # round-robin, OFDM_BENCH_BACKEND=gloo replaces RCCL (which refuses two
    # ranks on one GPU)
    have = torch.cuda.device_count()
    if os.environ.get("OFDM_BENCH_SHARE_GPU") == "1":
        local = local % max(1, have)
    elif local >= have:
        log(f"error: rank {rank} needs GPU {local} but only {have} visible")
        sys.exit(2)
    backend = os.environ.get("OFDM_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.mode == "split":
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    F, S, R, C, prefix = args.frames, args.S, args.R, args.C, args.prefix
    K = C - 1
    Q = F * (S - 1)  # data symbols per GPU per step
    import numpy as np
    rng = np.random.default_rng(args.seed)
    a = np.float32(0.70710678)
    X = torch.from_numpy((rng.choice([-a, a], K) + 1j * rng.choice([-a, a], K))
                         .astype(np.complex64)).to(dev)

    if args.mode == "split":
        return bench_split(args, X, dev, world, rank, barrier)
    if args.mode == "pcie":
        return bench_pcie(args, X, dev, world, rank, barrier)

    freq = args.mode == "freq"
    if freq:
        prefix = args.prefix = 0
    t = time.perf_counter()
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=args.seed, frame0=rank * F,
                           noise_std=args.noise, freq_domain=freq)
    ws = ofdm.workspace(F, S, R, C, dev)
    # the warm-up steps write out_w, the timed steps `out` (NaN-filled here,
    # before the warm-up, so nothing runs between the warm-up and the timed
    # loop): the timed steps recompute the warm-up's output from the same
    # input, so their last output must equal out_w bit for bit -- a check of
    # the one-launch kernel's inter-workgroup estimate hand-off on the
    # credited run itself
    out_w = ofdm.c64((F, S - 1, K), dev)
    out = ofdm.c64((F, S - 1, K), dev)
    out.fill_(float("nan"))
    torch.cuda.synchronize()
    log(f"[rank {rank}] synthesised {iq.numel() * 8 / 1e9:.1f} GB in {time.perf_counter() - t:.1f} s")

    stream = torch.cuda.current_stream()
    one = args.flow == "one" or (args.flow == "auto" and not freq and C == 1024)
    if one and (freq or C != 1024):
        raise SystemExit("--flow one: C = 1024, time domain only")

    # Two HIP events per step on the launch stream: after the estimate (LS)
    # and after the combine (MRC).  The LS of step i is timed from step i-1's
    # end event (one event before the loop for i = 0), so no event sits
    # between two steps' kernels beyond the one the MRC timing needs.
    # One-launch flow: the step is ofdm_frame_demod (k_demod_td<C>, LS and
    # MRC in one grid), timed from the previous step's end event.
    def step(evs=None, out=out):
        if one:
            ofdm.frame_demod(iq, X, prefix, ws=ws, out=out, stream=stream)
            if evs:
                evs[2].record(stream)
            return
        if freq:
            ofdm.frame_estimate_freq(iq, X, ws, stream)
        else:
            ofdm.frame_estimate(iq, X, prefix, ws, stream)
        if evs:
            evs[1].record(stream)
        if freq:
            ofdm.frame_combine_freq(iq, ws, out, stream)
        else:
            ofdm.frame_combine(iq, prefix, ws, out, stream)
        if evs:
            evs[2].record(stream)

    # the timing events exist before the warm-up and the warm-up's output is
    # checked after the timed loop: between the warm-up and the timed steps
    # only the contract's synchronize + barrier run, so the GPU is not left
    # idle for milliseconds (a fresh idle period restarts the clock's
    # response to load)
    events = [[None] + [torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    ev0 = torch.cuda.Event(enable_timing=True)
    for i in range(args.steps):
        events[i][0] = ev0 if i == 0 else events[i - 1][2]
    for _ in range(max(1, args.warmup)):
        step(out=out_w)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    errs_warm = int(ofdm.count_symbol_errors(out_w, S, seed=args.seed, frame0=rank * F).item())

    ls_ms = None if one else sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    mrc_all = sorted(e[0 if one else 1].elapsed_time(e[2]) for e in events)
    mrc_ms = sum(mrc_all) / args.steps
    mrc_median = mrc_all[len(mrc_all) // 2]
    errs = int(ofdm.count_symbol_errors(out, S, seed=args.seed, frame0=rank * F).item())
    same = bool(torch.equal(out, out_w))
    del out_w
    torch.cuda.empty_cache()

    # same-box context, after the timed loop (never inside it): the HBM copy /
    # read ceilings of this box, and the effective clock of the timed kernel
    # from its diagnostic build on the same batch
    box = box_probe(ofdm, torch, dev, stream) if not args.no_box else None
    clock = None
    if not args.no_box:
        ws_d = ofdm.workspace(F, S, R, C, dev)
        out_d = ofdm.c64((F, S - 1, K), dev)

        def step_diag():
            if one:
                ofdm.frame_demod(iq, X, prefix, ws=ws_d, out=out_d, stream=stream)
            else:
                ofdm.frame_estimate(iq, X, prefix, ws_d, stream)
                ofdm.frame_combine(iq, prefix, ws_d, out_d, stream)
        clock = clock_probe(step_diag, None if freq else DIAG_TAG.get(C), ofdm, torch, stream,
                            save=args.stamps_out)
        del ws_d, out_d
        torch.cuda.empty_cache()

    # per-rank spread (a SCALE shortfall points at a slow rank or at skew)
    rank_vals = [elapsed, mrc_ms, box["box_copy_GBps"] if box else float("nan"),
                 clock["effective_GHz_median"] if clock else float("nan")]
    stats = torch.tensor([elapsed, float(errs), float(errs_warm), 0.0 if same else 1.0],
                         dtype=torch.float64, device=dev)
    per_rank = None
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, errs, errs_warm, same = float(mx[0]), int(tot[1]), int(tot[2]), float(tot[3]) == 0.0
        rv = torch.tensor(rank_vals, dtype=torch.float64, device=dev)
        lo, hi = rv.clone(), rv.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        names = ["step_ms", "kernel_ms", "box_copy_GBps", "effective_GHz"]
        scale = [1e3 / args.steps, 1.0, 1.0, 1.0]
        fin = lambda v: v if v == v else None  # NaN (a probe that did not run) -> null: strict JSON
        per_rank = {n: {"min": fin(float(lo[i]) * scale[i]), "max": fin(float(hi[i]) * scale[i])}
                    for i, n in enumerate(names)}
    failed = not same or errs > 0
    if failed:
        log(f"CHECK FAILURE: timed output equals warm-up: {same}, QPSK errors on the timed output: {errs}")

    dom = "frequency-domain symbols (FFT upstream)" if freq else "time-domain IQ"
    cfg = {"workload": f"OFDM uplink LS+MRC, {dom} in HBM, {F} frames x {S} symbols "
                       f"(1 pilot + {S - 1} data) x {R} antennas x {C} subcarriers per GPU",
           "domain": "freq" if freq else "time",
           "R": R, "C": C, "S": S, "prefix": prefix, "frames_per_gpu": F,
           "data_symbols_per_gpu": Q, "global_data_symbols": Q * world,
           "flow": "one-launch" if one else "two-launch",
           "parallelism": f"frame-sharded x{world}, no collective"}
    b_sym = R * C * 8 + K * 8
    kern = {1024: "k_mrc_td1024_hlds", 2048: "k_mrc_td2048", 4096: "k_mrc_td4096h", 1536: "k_mrc_td1536", 3072: "k_mrc_td3072", 6144: "k_mrc_td6144", 512: "k_mrc_td512", 256: "k_mrc_td256", 128: "k_mrc_td128"}.get(C)
    mrc_name = f"{kern} (FFT+MRC+normalise+rotate)" if kern else "k_mrc_any (mixed-radix FFT+MRC+normalise+rotate)"
    if freq:
        mrc_name = "k_mrc_freq_frames (MRC+normalise+rotate)" if C >= 512 else "k_mrc_freq (MRC+normalise+rotate)"
    bytes_launch = Q * b_sym
    if one:  # + the pilot symbol and pilot vector per frame
        mrc_name = f"k_demod_td{C} (LS + FFT+MRC+normalise+rotate, one launch)"
        bytes_launch += F * (R * C * 8 + K * 8)
    achieved = bytes_launch / (mrc_ms * 1e-3) / 1e9
    build = ofdm.build_id()
    traffic, tsrc = pmc_traffic(args.pmc, cfg, build)
    step_bytes = F * S * R * C * 8 + Q * K * 8
    result = {
        "metric": "OFDM symbols/s (LS+MRC) at 1024 subcarriers x 64 ant; achieved HBM GB/s vs peak",
        "value": Q * world / (elapsed / args.steps),
        "unit": "symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated Rayleigh channel, QPSK, sigma=%g)" % args.noise,
        "config": cfg,
        "roofline": {"kernel": mrc_name, "bound": "hbm",
                     "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "traffic_source": tsrc,
                     "bytes_per_launch": bytes_launch, "avg_launch_ms": mrc_ms,
                     "median_launch_ms": mrc_median,
                     "box_copy_GBps": box["box_copy_GBps"] if box else None,
                     "frac_of_box_copy": achieved / box["box_copy_GBps"] if box else None,
                     "box_read_GBps": box["box_read_GBps"] if box else None,
                     "frac_of_box_read": achieved / box["box_read_GBps"] if box else None,
                     "box_probe": box["box_probe"] if box else None},
        "build_id": build,
        "clock": clock,
        "stages_ms": {"demod_one_launch": mrc_ms} if one else {"estimate_ls": ls_ms, "combine_mrc": mrc_ms},
        "step_algorithmic_GBps": step_bytes / (elapsed / args.steps) / 1e9,
        "per_rank": per_rank,
        "check": {"qpsk_symbol_errors": errs, "timed_equals_warmup": same,
                  "qpsk_symbol_errors_warmup": errs_warm,
                  "checked_output": "the last timed step's (its buffer NaN-filled before the warm-up)"},
        "cpu_baseline": None,
    }
    if failed:  # a broken run never yields a throughput that counts
        result["status"] = "CHECK_FAILED"
        result["value"] = None
        if rank == 0:
            print(json.dumps(result), flush=True)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(1)
    if world == 1 and not freq and not args.no_mode_a:
        del iq
        torch.cuda.empty_cache()
        result["mode_a"] = mode_a(args, X, ofdm, torch, dev, stream)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, X, ofdm, torch, dev)
        result["speedup_vs_cpu_baseline"] = result["value"] / result["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def mode_a(args, X, ofdm, torch, dev, stream):
    """Supplementary, outside the headline: the same frames in the frequency
    domain (FFT upstream), LS + MRC alone (SURVEY.md 8(d) mode A; DESIGN.md
    4.3) -- the north-star kernels k_ls_freq + k_mrc_freq_frames on the same
    shape, HIP events on the launch stream; `python bench.py --mode freq` is
    the full line."""
    F, S, R, C = args.frames, args.S, args.R, args.C
    K, Q = C - 1, args.frames * (args.S - 1)
    Y = ofdm.synth_frames(F, S, R, C, X, seed=args.seed, noise_std=args.noise, freq_domain=True)
    ws = ofdm.workspace(F, S, R, C, dev)
    out = ofdm.c64((F, S - 1, K), dev)
    steps = max(3, args.steps // 2)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for i in range(-1, steps):
        e = evs[i] if i >= 0 else None
        if e:
            e[0].record(stream)
        ofdm.frame_estimate_freq(Y, X, ws, stream)
        if e:
            e[1].record(stream)
        ofdm.frame_combine_freq(Y, ws, out, stream)
        if e:
            e[2].record(stream)
    torch.cuda.synchronize()
    errs = int(ofdm.count_symbol_errors(out, S, seed=args.seed).item())
    step_ms = sum(e[0].elapsed_time(e[2]) for e in evs) / steps
    mrc_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / steps
    achieved = Q * (R * C * 8 + K * 8) / (mrc_ms * 1e-3) / 1e9
    del Y, ws, out
    torch.cuda.empty_cache()
    return {"workload": f"the same {F} frames in the frequency domain (FFT upstream): LS + MRC alone",
            "value": Q / (step_ms * 1e-3), "unit": "symbols/s", "ms_per_step": step_ms, "steps": steps,
            "roofline": {"kernel": "k_mrc_freq_frames (MRC+normalise+rotate)", "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "avg_launch_ms": mrc_ms},
            "check": {"qpsk_symbol_errors": errs}}


def bench_pcie(args, X, dev, world, rank, barrier):
    """PCIe-inclusive receiver: --frames frames in page-locked HOST memory
    (what the ShMemSymBuff ring or a capture file hands over) streamed through
    ofdm_pipeline (chunk frames per slot, --depth slots; H2D, fused LS+MRC and
    D2H of the outputs on three HIP streams).  value = data symbols/s with
    the PCIe transfers included; pcie.h2d_GBps_copy_only = the same bytes
    copied with nothing else running (the bound of this mode)."""
    import torch
    import torch.distributed as dist
    import ofdm_lsmrc as ofdm
    F, S, R, C, prefix = args.frames, args.S, args.R, args.C, args.prefix
    K = C - 1
    Q = F * (S - 1)
    iq_d = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=args.seed, frame0=rank * F,
                             noise_std=args.noise)
    iq = torch.empty(iq_d.shape, dtype=iq_d.dtype, pin_memory=True)
    iq.copy_(iq_d)
    del iq_d
    out = torch.empty((F, S - 1, K), dtype=torch.complex64, pin_memory=True)
    torch.cuda.synchronize()
    in_bytes = iq.numel() * 8
    # copy-only bound: the same bytes H2D in chunk-sized copies, nothing else running
    scratch = torch.empty(args.chunk * S * R * (C + prefix), dtype=torch.complex64, device=dev)
    flat = iq.view(-1)
    n_el = scratch.numel()
    for _ in range(2):  # the second pass is timed
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for lo in range(0, flat.numel(), n_el):
            hi = min(lo + n_el, flat.numel())
            scratch[:hi - lo].copy_(flat[lo:hi], non_blocking=True)
        torch.cuda.synchronize()
        copy_s = time.perf_counter() - t0
    del scratch
    pipe = ofdm.Pipeline(S, R, C, X, prefix, chunk_frames=args.chunk, depth=args.depth)
    for _ in range(max(1, args.warmup)):
        pipe.demod(iq, out)
    pipe.sync()
    errs = int(ofdm.count_symbol_errors(out.to(dev), S, seed=args.seed, frame0=rank * F).item())
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.demod(iq, out)
    pipe.sync()
    elapsed = time.perf_counter() - t0
    barrier()
    if world > 1:
        mx = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[0])
    pipe.close()
    per_step = elapsed / args.steps
    result = {
        "metric": "OFDM symbols/s (LS+MRC) at 1024 subcarriers x 64 ant, PCIe-inclusive "
                  "(host-resident IQ and outputs)",
        "value": Q * world / per_step,
        "unit": "symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": per_step * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated, staged to page-locked host memory)",
        "config": {"workload": f"ofdm_pipeline: {F} host frames x {S} symbols x {R} antennas x "
                               f"{C} subcarriers per GPU, {args.chunk} frames/slot, "
                               f"{args.depth} slots",
                   "R": R, "C": C, "S": S, "prefix": prefix, "frames_per_gpu": F,
                   "chunk_frames": args.chunk, "depth": args.depth,
                   "parallelism": f"frame-sharded x{world}, no collective"},
        "pcie": {"h2d_GBps_pipeline": in_bytes / per_step / 1e9,
                 "h2d_GBps_copy_only": in_bytes / copy_s / 1e9,
                 "d2h_GBps_pipeline": Q * K * 8 / per_step / 1e9,
                 "frac_of_copy_only": copy_s / per_step},
        "check": {"qpsk_symbol_errors": errs},
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_split(args, X, dev, world, rank, barrier):
    """configs[4]: every rank holds all frames of ITS --R antennas (global
    antennas rank*R ...); step = SplitPipeline.run (one partial LS over the
    batch, all_reduce of |H|^2, then per chunk the partial FFT+MRC,
    reduce_scatter of the numerators over RCCL and the finalise of the rank's
    slice), chunked so the collectives overlap the next chunk's kernels.  value = data symbols demodulated per second (every
    rank covers the same symbols; the antenna count grows with N)."""
    import torch
    import torch.distributed as dist
    import ofdm_lsmrc as ofdm
    import antenna_split
    F, S, R, C, prefix = args.frames, args.S, args.R, args.C, args.prefix
    K = C - 1
    Q = F * (S - 1)
    t = time.perf_counter()
    iq = ofdm.synth_frames(F, S, R, C, X, prefix=prefix, seed=args.seed, r0=rank * R,
                           noise_std=args.noise)
    out = ofdm.c64((F, S - 1, K), dev)
    pipe = antenna_split.SplitPipeline(F, S, R, C, prefix, dev, chunk_frames=args.chunk)
    torch.cuda.synchronize()
    log(f"[rank {rank}] synthesised {iq.numel() * 8 / 1e9:.1f} GB in {time.perf_counter() - t:.1f} s")
    for _ in range(max(1, args.warmup)):
        pipe.run(iq, X, out)
    # the timed steps write every output position on exactly one rank (its
    # reduce-scatter slice), so `out` is zeroed first and gathered ONCE after
    # the timed loop: what is checked below is what the timed steps computed
    out.zero_()
    torch.cuda.synchronize()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.run(iq, X, out)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    if world > 1:
        mx = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[0])
        dist.all_reduce(torch.view_as_real(out))  # the gather: each position is non-zero on one rank only
    torch.cuda.synchronize()
    errs = int(ofdm.count_symbol_errors(out, S, seed=args.seed).item()) if rank == 0 else 0
    check = {"qpsk_symbol_errors": errs}
    if rank == 0:
        check["vs_full_receiver"] = split_vs_full(ofdm, torch, X, out, F, S, R * world, C, prefix, args)

    # stage times of one more (untimed) step, per rank, then max over ranks:
    # partial LS / partial FFT+MRC / finalise on the compute stream, the
    # communication the overlap left exposed, and the collectives alone
    barrier()
    stages = pipe.profile_step(iq, X, out, stream=torch.cuda.current_stream())
    keys = sorted(k for k, v in stages.items() if isinstance(v, float))
    if world > 1:
        v = torch.tensor([stages[k] for k in keys], dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        stages.update({k: float(v[i]) for i, k in enumerate(keys)})
    stages["reduction"] = "max over ranks" if world > 1 else "one rank"

    # roofline of the dominant kernel: the partial FFT+MRC over the whole
    # local batch, HIP events on its stream (outside the timed region)
    stream = torch.cuda.current_stream()
    _, ws = ofdm.frame_ls_partial(iq, X, prefix)
    num = ofdm.c64((F, S - 1, K), dev)
    reps = 5
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ofdm.frame_mrc_partial(iq, ws, prefix, num=num)
    evs[0].record(stream)
    for i in range(reps):
        ofdm.frame_mrc_partial(iq, ws, prefix, num=num)
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    mrc_all = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(reps))
    mrc_ms = sum(mrc_all) / reps
    mrc_median = mrc_all[reps // 2]
    b_sym = R * C * 8 + K * 8
    achieved = Q * b_sym / (mrc_ms * 1e-3) / 1e9
    kern = {1024: "k_mrc_td1024_hlds", 2048: "k_mrc_td2048", 4096: "k_mrc_td4096h", 1536: "k_mrc_td1536", 3072: "k_mrc_td3072", 6144: "k_mrc_td6144", 512: "k_mrc_td512", 256: "k_mrc_td256", 128: "k_mrc_td128"}.get(
        C, "k_mrc_any")
    result = {
        "metric": "OFDM symbols/s (LS+MRC) at 1024 subcarriers x 64 ant; achieved HBM GB/s vs peak",
        "value": Q / (elapsed / args.steps),
        "unit": "symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated Rayleigh channel, QPSK, sigma=%g)" % args.noise,
        "config": {"workload": f"OFDM uplink LS+MRC, antenna split: {F} frames x {S} symbols x "
                               f"{R * world} antennas ({R} per GPU) x {C} subcarriers",
                   "R_per_gpu": R, "R_total": R * world, "C": C, "S": S, "prefix": prefix,
                   "frames": F, "data_symbols": Q, "chunk_frames": args.chunk,
                   "parallelism": f"antenna-split x{world}, all_reduce(|H|^2) + "
                                  f"reduce_scatter(numerators) over RCCL"},
        "roofline": {"kernel": f"{kern} partial numerators (FFT+MRC)", "bound": "hbm",
                     "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "bytes_per_launch": Q * b_sym, "avg_launch_ms": mrc_ms,
                     "median_launch_ms": mrc_median},
        "stages_ms": stages,
        "build_id": ofdm.build_id(),
        "check": check,
        "cpu_baseline": None,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.destroy_process_group()


def split_vs_full(ofdm, torch, X, out, F, S, R_total, C, prefix, args):
    """Frames 0 and F-1 of the gathered antenna-split output against the
    single-GPU receiver (ofdm.frame_demod, parity-tested against the oracle in
    tests/) on ALL R_total antennas of the same frames, re-synthesised on this
    rank: a wrong collective order or slice shows up here as a parity failure,
    not only as a speed number.  Tolerance: north_star's 1e-5 (the split sums
    the antennas per rank, then across ranks)."""
    import numpy as np
    worst_n, worst_e = 0.0, 0.0
    for f in sorted({0, F - 1}):
        full = ofdm.synth_frames(1, S, R_total, C, X, prefix=prefix, seed=args.seed, frame0=f,
                                 noise_std=args.noise)
        ref = ofdm.frame_demod(full, X, prefix)[0].cpu().numpy().astype(np.complex128).ravel()
        got = out[f].cpu().numpy().astype(np.complex128).ravel()
        del full
        nrel = float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))
        rms = float(np.sqrt(np.mean(np.abs(ref) ** 2)))
        erel = float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), rms)))
        worst_n, worst_e = max(worst_n, nrel), max(worst_e, erel)
    torch.cuda.empty_cache()
    ok = bool(np.isfinite(worst_n) and worst_n <= 1e-5 and worst_e <= 1e-5)
    if not ok:
        log(f"SPLIT PARITY FAILURE: norm-rel {worst_n:.3e}, elem-rel {worst_e:.3e} vs the full receiver")
    return {"frames": sorted({0, F - 1}), "antennas": R_total, "norm_rel": worst_n, "max_elem_rel": worst_e,
            "tolerance": 1e-5, "ok": ok}


if __name__ == "__main__":
    main()
