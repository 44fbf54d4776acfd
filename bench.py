#!/usr/bin/env python3
"""Benchmark: acquire decisions/s of the MI355X token-bucket engine (BASELINE.json metric).

Workload (BASELINE.json configs[1]): TokenBucket over 100M keys,
uniform keys, batches of 2^26 requests, permits = 1, TokenLimit 10, 1 token / 1 s,
batch b spans 10 ms of injected time.  A "step" is one batch: the full decision
pipeline (partition, fold, un-partition) over 2^26 requests already resident in HBM.

Multi-GPU (one rank per GPU): keys are hash-partitioned, each rank owns 100M / N keys
in its own HBM and decides its own 2^26-request batches (no data-path collective: weak
scaling).  value = all ranks' decisions / max-over-ranks time.  Under torchrun the ranks
come from the environment; `bench.py --gpus N` without one starts the N ranks itself
(torch.distributed.run as a child process, from a parent that never touches the GPU)
and exits with its status.  A run whose world size is not N exits non-zero instead of
printing a line.

Also reported: per-stage device time, the roofline of the dominant kernel (HIP events
on the engine stream; for the pipelined engine, over a serial replay of the same timed
batches, since overlapped stages share the chip), and the CPU baseline (the C
restatement of the reference script, oracle/tb_ref.c, on a bounded sample of the same
trace).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_kinds import (cpu_model, gather_floats, mark, pmc_workload, reduce_max,  # noqa: E402
                         run_fingerprint, write_fingerprint)

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED_B = 0x5EED000B
SEED_C = 0x5EED000C
SEED_A = 0x5EED0001
T0_US = 1_760_000_000_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the schedule tools/pmc_passes.sh measures, so that a run without flags
    # matches profiles/pmc_summary.json's fingerprint and carries its PMC traffic
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("uniform", "zipf", "queue", "approx", "testapp"),
                    default="uniform",
                    help="uniform: config B (the headline); zipf: config C's per-GPU slice; "
                         "queue: config D (TokenBucketWithQueue); approx: config E (two-tier); "
                         "testapp: config A (the TestApp limiter: 10k keys, 1M requests per 2 s)")
    ap.add_argument("--keys", type=int, default=None,
                    help="total keys (uniform, default 1e8) / keys per GPU (zipf, default 1.25e8)")
    ap.add_argument("--zipf-s", type=float, default=1.1)
    ap.add_argument("--route", choices=("pre", "timed"), default="pre",
                    help="N > 1: route each step's global requests to their owners before the timed "
                         "region (ingest partitioned) or inside every timed step")
    ap.add_argument("--approx-mode", choices=("node", "clients"), default="node",
                    help="config E with N > 1: the node as one client (RCCL all-reduce of the counts, "
                         "the north star's global tier; default) or every rank a client (all-gather); "
                         "the other mode's refresh epoch is timed after the timed region too")
    ap.add_argument("--owner-map", choices=("hash", "balanced"), default=None,
                    help="N > 1: owner of a key = the hash partition (SURVEY.md §8e) or a balanced owner map "
                         "built from step 0's all-reduced virtual-node loads (DESIGN.md §7; default for zipf)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="zipf, one GPU: emulate config C's owners at this many GPUs one at a time "
                         "(bench_emul.py; the line is marked as an emulation)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0 with the gloo backend (the "
                         "device path's collectives stage through host memory); the line is marked "
                         "'rehearsal' and its times are not a scaling measurement")
    ap.add_argument("--batch", type=int, default=None, help="requests per batch (default 2^26; testapp 1M)")
    ap.add_argument("--interval-us", type=int, default=None,
                    help="injected time per batch (default 10 ms; 1 ms for queue)")
    ap.add_argument("--token-limit", type=int, default=None,
                    help="TokenLimit (default 10; 4 for queue, 100 for approx)")
    ap.add_argument("--queue-limit", type=int, default=16)
    ap.add_argument("--no-fuse-tick", action="store_true",
                    help="config D: replenish tick as its own pass (tbe_refresh_device) instead of "
                         "fused into the batch's fold (A/B)")
    ap.add_argument("--no-drain-variant", action="store_true",
                    help="config D: skip the second schedule whose ticks grant (draining block)")
    ap.add_argument("--settle-s", type=float, default=0.0,
                    help="seconds to wait before the first allocation (lets background device-memory "
                         "work left by an earlier process finish; reported in the line)")
    ap.add_argument("--engine-first", action="store_true",
                    help="config D: create the engine before generating the inputs (A/B; round 5's order)")
    ap.add_argument("--drain-marked", action="store_true",
                    help="config D: put the PMC window markers around the draining schedule's timed "
                         "batches instead of the headline's (tools/pmc_passes.sh, run queue_draining)")
    ap.add_argument("--tokens-per-period", type=int, default=1)
    ap.add_argument("--period-ticks", type=int, default=None,
                    help="ReplenishmentPeriod in 100 ns ticks (default 1 s; approx: one batch interval)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="approximate CPU-baseline budget (0 disables)")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--timed-stage-events", action="store_true",
                    help="record the stage events in the timed (pipelined) engine too (A/B: each "
                         "event record costs the stream a bubble; by default the stage times come "
                         "from the serial replay alone)")
    ap.add_argument("--no-host-buffer", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) rate, e.g. under rocprofv3 so the "
                         "kernel statistics cover the timed batches only")
    ap.add_argument("--no-pack", action="store_true",
                    help="wide pass records even where the packed 8-byte form applies (A/B)")
    ap.add_argument("--no-hot", action="store_true", help="no hot-key runs (A/B)")
    ap.add_argument("--no-narrow", action="store_true",
                    help="4-byte replies even where TokenLimit <= 127 allows 1-byte ones (A/B)")
    ap.add_argument("--no-sparse", action="store_true",
                    help="skip the batch-size sweep (2^14 .. 2^26-request batches over config B's keys)")
    ap.add_argument("--sweep-log2", default=None,
                    help="comma-separated log2 batch sizes of the sweep (default 14,16,...,26)")
    ap.add_argument("--sweep-zipf", action="store_true",
                    help="the sweep's batches draw Zipf(--zipf-s) keys instead of uniform ones (A/B)")
    ap.add_argument("--no-strdir", action="store_true",
                    help="skip the string-key directory leg (config B batches as key text)")
    ap.add_argument("--unscatter-all", action="store_true",
                    help="plain last-pass records, every pass's permutation and un-partition "
                         "(TBE_FLAG_UNSCATTER_ALL; A/B of the fold records and k_unrank)")
    ap.add_argument("--hist-records", action="store_true",
                    help="the second pass's histogram reads the first pass's records, not the "
                         "one-byte digit stream (TBE_FLAG_HIST_RECORDS; A/B)")
    ap.add_argument("--rerank", action="store_true",
                    help="the final un-partition re-ranks pass 0's tiles from one-byte digits instead "
                         "of gathering through pass 0's permutation (TBE_FLAG_RERANK; A/B of k_unrank)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one stream per batch: no overlap of batch b+1's partition with batch b's fold (A/B)")
    args = ap.parse_args()
    testapp = args.workload == "testapp"
    if args.batch is None:
        args.batch = 1_000_000 if testapp else 1 << 26
    if args.interval_us is None:
        args.interval_us = {"queue": 1_000, "testapp": 2_000_000}.get(args.workload, 10_000)
    if args.token_limit is None:
        args.token_limit = {"queue": 4, "approx": 100, "testapp": 20}.get(args.workload, 10)
    if testapp and args.tokens_per_period == 1:
        args.tokens_per_period = 10    # TokenLimit 20, 10 / s
    if args.period_ticks is None:
        args.period_ticks = args.interval_us * 10 if args.workload == "approx" else 10_000_000
    if args.workload == "approx" and args.tokens_per_period == 1:
        args.tokens_per_period = 10
    if args.owner_map is None:
        args.owner_map = "balanced" if args.workload == "zipf" else "hash"
    return args


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) outside torchrun: run this script as N ranks under
    torch.distributed.run, one per GPU, and return its exit status.  This process makes
    no GPU call (torch.cuda.device_count() does not initialise the runtime on this image)
    and starts the ranks as a child process, never by exec."""
    if not args.share_device:
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dist_setup(args):
    """(world, rank, local_rank, dist, device) of this rank; exits non-zero when the
    world size is not --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: world size {world} != --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    dist = world > 1
    if dist:
        print(f"bench.py: rank {rank} of {world}", file=sys.stderr, flush=True)
    gpu = 0 if args.share_device else local_rank
    if dist and args.share_device:
        # gloo first: both ranks have reported in before either touches the device
        import torch.distributed as td
        td.init_process_group("gloo")
    torch.cuda.set_device(gpu)
    if dist:
        import torch.distributed as td
        if not args.share_device:
            td.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        if td.get_world_size() != args.gpus:
            print(f"bench.py: process group has {td.get_world_size()} ranks, --gpus {args.gpus}",
                  file=sys.stderr)
            sys.exit(2)
    return world, rank, local_rank, dist, torch.device("cuda", gpu)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.settle_s > 0:
        time.sleep(args.settle_s)
    world, rank, local_rank, dist, dev = dist_setup(args)
    if dist:
        import torch.distributed as td

    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi

    lib = _capi.load()
    lib.tbe_gen_batch_device.restype = ctypes.c_int
    lib.tbe_gen_batch_device.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_int32] * 2 + \
        [ctypes.c_int64] * 2 + [ctypes.c_void_p] * 4
    if args.emulate_world:
        import bench_emul
        if args.workload != "zipf" or world != 1:
            print("bench.py: --emulate-world needs --workload zipf on one GPU", file=sys.stderr)
            sys.exit(2)
        print(json.dumps(bench_emul.run(args, lib, dev)), flush=True)
        return
    if args.workload in ("queue", "approx"):
        import bench_kinds
        line = bench_kinds.run(args, lib, dev, world, rank, dist)
        if args.share_device:
            line["rehearsal"] = REHEARSAL_NOTE
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            td.destroy_process_group()
        return

    # Key space and ownership.  One GPU owns every key, so the generated
    # ids are its bucket ids.  With N ranks, every rank draws its share of ONE global
    # request stream (uniform over 1e8 keys, or Zipf(1.1) over 1.25e8 * N keys for config C),
    # and the requests go to their owners, owner = mix64(key) >> (64 - log2 N), whose key
    # directories turn them into dense bucket ids (cluster.route_requests: stable
    # partition + RCCL all-to-all + directory, all in HBM).  --route pre (default) routes
    # before the timed region, i.e. ingest arrives partitioned (the benchmark mode of
    # §8e); --route timed keeps the exchange, the directory and the replies' way back in
    # every timed step.  Either way the hot keys of a Zipf stream load their owners
    # unevenly, and the slowest rank sets the time.
    if args.workload == "zipf":
        keys_total = (args.keys or 125_000_000) * world
    else:
        keys_total = args.keys or (10_000 if args.workload == "testapp" else 100_000_000)
    from distributedratelimiting.redis_amd import cluster
    n = args.batch
    total_steps = args.warmup + args.steps
    routed = dist and args.workload != "testapp"
    if routed:   # the device path orders the engine on a real stream (cluster.device_stream)
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    seed = {"zipf": SEED_C, "testapp": SEED_A}.get(args.workload, SEED_B)
    gen_stream = torch.cuda.current_stream(dev).cuda_stream or None

    def gen_batch(s):   # this rank's share of the global stream at step s
        g0 = (s * world + rank) * n
        k = torch.empty(n, dtype=torch.int64, device=dev)
        p = torch.empty(n, dtype=torch.int32, device=dev)
        t = torch.empty(n, dtype=torch.int64, device=dev)
        assert lib.tbe_gen_batch_device(seed, keys_total, g0, n, 1, 1, T0_US + s * args.interval_us,
                                        args.interval_us, k.data_ptr(), p.data_ptr(), t.data_ptr(), gen_stream) == 0
        if args.workload == "zipf":
            assert lib.tbe_gen_zipf_keys_device(seed, keys_total, args.zipf_s, g0, n, k.data_ptr(), gen_stream) == 0
        return k, p, t

    # the owner map (N > 1): the hash partition, or balanced from step 0's virtual-node loads
    # summed over the ranks, so every rank builds the same map before any key is routed
    omap = None
    if routed and args.owner_map == "balanced":
        loads = cluster.vnode_loads(gen_batch(0)[0])
        cluster._all_reduce_sum(loads)
        omap = cluster.balanced_owner_map(loads.cpu().numpy(), world, n_keys=keys_total)
    keys_local = cluster.keys_per_rank(keys_total, world, owner_map=omap)
    # --route timed: the directory's overflow check must not synchronise inside a step
    directory = cluster.DeviceDirectory(keys_local, device=dev.index, strict=args.route != "timed") \
        if routed else None
    bufs, raw = [], []
    # generated on the current stream: the routing kernels run on it too (a torch stream does
    # not wait for the legacy NULL stream)
    for s in range(total_steps):
        k, p, t = gen_batch(s)
        if routed and args.route == "pre":
            (lk, lp, lt), _ = cluster.route_requests(k, p, t, directory, owner_map=omap)
            bufs.append((lk, lp, lt))
        elif routed:
            raw.append((k, p, t))
        else:
            bufs.append((k, p, t))
    torch.cuda.synchronize()
    sizes = [b[0].numel() for b in bufs] or [n]
    m_max = max(sizes)
    # Stage events in the timed engine only when no serial replay follows to take the stage
    # times from (routed batches, or no pipeline): an event record between two kernels leaves
    # the stream idle for several microseconds (profiles/r05n_*), ~14 of them per batch.
    replay = not args.no_pipeline and not args.no_stage_timing and not (routed and args.route != "pre")
    eng = TokenBucketEngine(keys_local, args.token_limit, args.tokens_per_period,
                            args.period_ticks, device=dev.index,
                            stage_timing=not args.no_stage_timing and (not replay or args.timed_stage_events),
                            max_batch=m_max,
                            pack=not args.no_pack, hot=not args.no_hot, narrow=not args.no_narrow,
                            pipeline=not args.no_pipeline, fold_records=not args.unscatter_all,
                            digit_stream=not args.hist_records, rerank=args.rerank)
    layout = eng.layout()
    if rank == 0:
        write_fingerprint(run_fingerprint(args, world, keys_local, layout))
    granted = torch.empty(m_max if not raw else n, dtype=torch.uint8, device=dev)
    remaining = torch.empty(m_max if not raw else n, dtype=torch.int32, device=dev)
    zkeys = [bufs[s][0].cpu().numpy().view(np.uint64) for s in range(min(2, len(bufs)))] \
        if args.workload == "zipf" and not routed else []
    cur = torch.cuda.current_stream(dev).cuda_stream

    def decide(lk, lp, lt):   # --route timed: the owner's engine on the routed requests
        g = torch.empty(lk.numel(), dtype=torch.uint8, device=dev)
        r = torch.empty(lk.numel(), dtype=torch.int32, device=dev)
        eng.acquire_batch_device(lk, lp, lt, g, r, stream=cur)
        return g, r

    def step(s):
        if raw:
            g, r = cluster.route_batch(decide, *raw[s], directory, owner_map=omap)
            granted.copy_(g)
            remaining.copy_(r)
        else:
            m = bufs[s][0].numel()
            eng.acquire_batch_device(*bufs[s], granted[:m], remaining[:m])

    for s in range(args.warmup):
        step(s)
    eng.synchronize()
    torch.cuda.synchronize()
    eng.stage_times()  # discard warm-up stage times

    mark(lib, 1, dev)     # profiling marker: the timed batches follow (outside the timing)
    if dist:
        td.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, total_steps):
        step(s)
    eng.synchronize()
    torch.cuda.synchronize()
    if dist:
        td.barrier()
    elapsed = time.perf_counter() - t0
    mark(lib, 2, dev)
    load = None
    if dist:
        elapsed = reduce_max(elapsed, dev)
        # requests each owner decided in the timed steps: max / mean = the hash partition's
        # imbalance (Zipf: the hot keys' owners)
        ev = gather_floats(float(sum(sizes[args.warmup:])), world, dev)
        load = {"per_rank_requests": ev.tolist(), "max_over_mean": round(float(ev.max() / ev.mean()), 4)}
    stages_overlapped = eng.stage_times()
    m_last = (raw[-1][0] if raw else bufs[total_steps - 1][0]).numel()
    grant_rate = float(granted[:m_last].float().mean().item())
    # SURVEY.md §8(d) B_alg of the last timed batch, measured: U = its distinct keys, W =
    # the distinct keys it wrote (granted at least once; a deny writes nothing, TB:225-236)
    last_keys = raw[-1][0] if raw else bufs[total_steps - 1][0]
    u_meas = int(torch.unique(last_keys).numel())
    w_meas = int(torch.unique(last_keys[granted[:m_last].bool()]).numel())
    step_alg = int(m_last * 25 + u_meas * 16 + w_meas * 16)
    uw_note = "U and W measured on the last timed batch"

    decisions = n * args.steps * world
    value = decisions / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- per-kernel times for the roofline.  A pipelined engine overlaps batch b+1's
    # partition with batch b's fold, so its per-stage event intervals include the time the
    # two share the chip.  Kernel durations are therefore taken from a serial replay (one
    # stream, pipeline off) of exactly the same warm-up + timed batches on a second engine,
    # right after the timed region; its replies must equal the pipelined run's.
    stages, replay_check = stages_overlapped, None
    line_read = line_written = None
    if replay and layout.get("pipeline"):
        eng.close()
        ser = TokenBucketEngine(keys_local, args.token_limit, args.tokens_per_period,
                                args.period_ticks, device=dev.index, stage_timing=True,
                                max_batch=n, pack=not args.no_pack, hot=not args.no_hot, narrow=not args.no_narrow,
                                pipeline=False, fold_records=not args.unscatter_all,
                            digit_stream=not args.hist_records, rerank=args.rerank)
        g2 = torch.empty_like(granted)
        r2 = torch.empty_like(remaining)
        for s in range(args.warmup):
            ser.acquire_batch_device(*bufs[s], g2[:sizes[s]], r2[:sizes[s]])
        ser.synchronize()
        ser.stage_times()
        g_all = [torch.empty(sizes[s], dtype=torch.uint8, device=dev) for s in range(args.warmup, total_steps)]
        mark(lib, 3, dev)     # profiling marker: the replay's timed batches follow (tools/prof_window.py)
        for i, s in enumerate(range(args.warmup, total_steps)):
            ser.acquire_batch_device(*bufs[s], g_all[i], r2[:sizes[s]])
        mark(lib, 4, dev)
        ser.synchronize()
        stages = ser.stage_times()
        replay_check = bool(torch.equal(g_all[-1][:m_last], granted[:m_last]) and
                            torch.equal(r2[:m_last], remaining[:m_last]))
        # U and W of every timed batch (the replay's grants equal the timed run's): the
        # step's B_alg is their mean, not just the last batch's (the table ages from
        # grant- to denial-dominated across the timed batches)
        uw = []
        lines = []   # 128-byte table lines (8 rows) touched / holding a written row, per batch
        for i, s in enumerate(range(args.warmup, total_steps)):
            k = bufs[s][0]
            kw = k[g_all[i].bool()]
            uw.append((int(torch.unique(k).numel()), int(torch.unique(kw).numel())))
            lines.append((int(torch.unique(k // 8).numel()), int(torch.unique(kw // 8).numel())))
        del g_all
        line_read = float(np.mean([a for a, _ in lines]))
        line_written = float(np.mean([b for _, b in lines]))
        u_mean = float(np.mean([u for u, _ in uw]))
        w_mean = float(np.mean([w for _, w in uw]))
        step_alg = int(n * 25 + u_mean * 16 + w_mean * 16)
        uw_note = (f"mean over the {len(uw)} timed batches: U {u_mean:.4g}, W {w_mean:.4g} "
                   f"(first {uw[0][1]}, last {uw[-1][1]} written keys)")
        u_meas, w_meas = int(round(u_mean)), int(round(w_mean))
        eng = ser

    # ---- roofline: the decision kernel -- the fold,
    # which reads and writes the table -- is the dominant kernel, and its `achieved` is the
    # step's algorithmic bytes B_alg (25 B per request + 16 B per distinct key read + 16 B
    # per key written) over the fold's average launch time.  The fold's own byte count
    # (records, replies and rows) is kept beside it as kernel_own_*; the stage with the most
    # device time is named too.
    roofline = None
    if stages and stages.get("fold", 0) > 0:
        passes = layout["passes"]
        launches = {"hist": passes, "colscan": passes, "scatter": passes, "bounds": 1, "fold": 1,
                    "unscatter": passes - (1 if layout.get("fold_records") else 0), "hot": 5}   # per step
        name = "fold"
        largest = max(stages, key=stages.get)
        per_launch_ms = stages[name] / (args.steps * launches[name])
        own_bytes = algorithmic_bytes(name, n, keys_local, passes, layout["packed"], u_meas,
                                      1 if layout.get("narrow") else 4, w_meas)
        achieved = step_alg / (per_launch_ms * 1e-3) / 1e9
        own_achieved = own_bytes / (per_launch_ms * 1e-3) / 1e9
        step_achieved = step_alg / (ms_per_step * 1e-3) / 1e9
        fp = run_fingerprint(args, world, keys_local, layout)
        w_pmc, pmc_why = pmc_workload(args.workload, fp)
        pmc = pmc_stage(w_pmc, name)
        if w_pmc is not None and pmc is None:
            pmc_why = f"no PMC bytes for the {name} stage"
        step_pmc = pmc_step_traffic(w_pmc)
        roofline = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": (round(pmc / launches[name], 1) if pmc is not None else None),
                    **({"traffic_null_reason": pmc_why} if pmc is None else {}),
                    "alg_bytes_per_launch": step_alg,
                    "alg_bytes_note": ("SURVEY.md §8(d) B_alg of the batch one fold launch decides: 25 B per "
                                       "request + 16 B per distinct key read + 16 B per distinct key written; "
                                       + uw_note),
                    "kernel_own_bytes": own_bytes,
                    "kernel_own_note": algorithmic_note(name, layout, u_meas, w_meas),
                    "kernel_own_frac": round(own_achieved / HBM_PEAK_GBS, 4),
                    "largest_stage": largest,
                    "largest_stage_ms_per_step": round(stages[largest] / args.steps, 4),
                    "distinct_keys_U": u_meas, "written_keys_W": w_meas,
                    "step_alg_bytes": step_alg,
                    "step_achieved": round(step_achieved, 1),
                    "step_frac": round(step_achieved / HBM_PEAK_GBS, 4),
                    "step_traffic": step_pmc,
                    **({"step_traffic_null_reason": pmc_why or "no step bytes in the PMC summary"}
                       if step_pmc is None else {}),
                    "traffic_source": PMC_SOURCE,
                    "fingerprint": fp,
                    "avg_launch_ms": round(per_launch_ms, 4),
                    "timing": ("serial replay of the timed batches (pipeline off), HIP events on the "
                               "engine stream" if replay_check is not None else
                               "HIP events on the engine stream over the timed region")}
        if name == "fold" and line_read is not None:
            # The fold's floor at the memory's own granularity: a 16-byte row costs its whole
            # 128-byte line, read if any row of the line is requested and written if any is
            # granted (nearly every line at config B's key/batch ratio), plus the records and
            # replies.  SURVEY §8(d) prices 16 B per distinct key instead.
            line_floor = int(round((line_read + line_written) * 128 +
                                   n * ((8 if layout["packed"] else 16) + (1 if layout.get("narrow") else 4))))
            roofline.update({
                "line_floor_bytes": line_floor,
                "line_frac": round(line_floor / (per_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "line_note": (f"128 B x (lines read {line_read:.4g} + lines written {line_written:.4g}, "
                              "per-batch means of the timed batches) + records and replies")})
        if replay_check is not None:
            if args.timed_stage_events:   # (the timed engine records stage events only then)
                roofline["overlapped_avg_launch_ms"] = round(
                    stages_overlapped.get(name, 0.0) / (args.steps * launches[name]), 4)
            roofline["replay_replies_identical"] = replay_check

    # config A is the reference's own per-request deployment: also time the host-buffer
    # entry point (the P/Invoke path: copy in, decide, copy out, synchronise) on the same
    # batches, after the timed region.  Reported beside `value`, never as it.
    # Config B gets the same check on three of its batches (pageable host buffers: the
    # PCIe-inclusive rate DESIGN.md §6 discusses).
    host_rate = host_rate_pinned = None
    if args.workload in ("testapp", "uniform") and rank == 0 and world == 1 and not args.no_host_buffer:
        timed_bufs = bufs[args.warmup:] if args.workload == "testapp" else bufs[args.warmup:args.warmup + 3]
        host = [tuple(x.cpu().numpy() for x in b) for b in timed_bufs]
        hb = TokenBucketEngine(keys_local, args.token_limit, args.tokens_per_period, args.period_ticks,
                               device=dev.index, max_batch=n)
        for k, p, t in host[:1]:
            hb.acquire_batch(k.view(np.uint64), p, t)
        t1 = time.perf_counter()
        for k, p, t in host[1:]:
            hb.acquire_batch(k.view(np.uint64), p, t)
        host_rate = round(n * (len(host) - 1) / (time.perf_counter() - t1), 1) if len(host) > 1 else None
        if len(host) > 1:
            # the same batches from page-locked buffers (tbe_alloc_host): DMA, no staging copy
            from distributedratelimiting.redis_amd.engine import PinnedArray
            pk, pp, pt = PinnedArray(n, np.uint64), PinnedArray(n, np.int32), PinnedArray(n, np.int64)
            pg, pr = PinnedArray(n, np.uint8), PinnedArray(n, np.int32)
            spent = 0.0
            for k, p, t in host[1:]:
                pk.array[:], pp.array[:], pt.array[:] = k.view(np.uint64), p, t
                t1 = time.perf_counter()
                hb.acquire_batch(pk.array, pp.array, pt.array, pg.array, pr.array)   # chunked, overlapped
                spent += time.perf_counter() - t1
            host_rate_pinned = round(n * (len(host) - 1) / spent, 1)
            for a in (pk, pp, pt, pg, pr):
                a.free()
        hb.close()

    # the string-key path: the same batches as key text
    # "user-<key>" through the device string directory, after the timed region
    strdir = None
    if args.workload == "uniform" and rank == 0 and world == 1 and not args.no_strdir:
        strdir = bench_strdir(bufs[:6], keys_local, dev)

    # batch sizes 2^14 .. 2^26 on the same key space; "sparse_batch" is
    # its 2^20 point (2^20 requests over 1e8 keys touch ~1% of the table's lines: the sparse
    # buckets go one wave each to k_fold_sparse, which gathers only their rows)
    sparse = sweep = None
    if args.workload == "uniform" and rank == 0 and world == 1 and not args.no_sparse:
        sizes = tuple(int(x) for x in args.sweep_log2.split(",")) if args.sweep_log2 else SWEEP_LOG2
        sweep = bench_batch_sweep(args, lib, keys_local, dev, sizes)
        sparse = next((x for x in sweep if x["batch"] == 1 << 20), None)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, keys_local, zkeys,
                           SEED_A if args.workload == "testapp" else SEED_B)

    if rank == 0:
        line = {
            "metric": "acquire decisions/sec (node) at 100M keys, 1/2/4/8 GPU; % HBM roofline",
            "value": round(value, 1),
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (Zipf(1.1) keys by rejection-inversion, splitmix64 counters, "
                     "generated in HBM)" if args.workload == "zipf" else
                     "synthetic (splitmix64 seeded trace generated in HBM)"),
            "config": {"workload": workload_name(args, n),
                       "keys_total": keys_total, "keys_per_gpu": keys_local, "batch_per_gpu": n,
                       "token_limit": args.token_limit, "tokens_per_period": args.tokens_per_period,
                       "period_ticks": args.period_ticks, "interval_us": args.interval_us,
                       "partitioning": ("one GPU owns every key" if world == 1 else
                                        (f"owner = mix64(key) >> (64 - log2 {world})" if omap is None else
                                         "owner = a balanced owner map (cluster.balanced_owner_map of step 0's "
                                         "all-reduced virtual-node loads)") +
                                        "; each rank draws its share of one global stream, routed to the owners "
                                        + ("before the timed region (ingest partitioned, no "
                                           "data-path collective timed)" if args.route == "pre" else
                                           "inside every timed step (RCCL all-to-all both ways)")),
                       "layout": layout},
            **({"rehearsal": REHEARSAL_NOTE} if args.share_device else {}),
            "grant_rate_last_batch": round(grant_rate, 4),
            **({"owner_load": load} if load is not None else {}),
            **({"host_buffer_decisions_per_s": host_rate} if host_rate is not None else {}),
            **({"host_buffer_pinned_decisions_per_s": host_rate_pinned}
               if host_rate_pinned is not None else {}),
            **({"string_directory": strdir} if strdir is not None else {}),
            **({"sparse_batch": sparse} if sparse is not None else {}),
            **({"batch_sweep": sweep} if sweep is not None else {}),
            "stage_ms_per_step": {k: round(v / args.steps, 4) for k, v in stages.items()},
            "stage_ms_per_step_overlapped": ({k: round(v / args.steps, 4)
                                              for k, v in stages_overlapped.items()}
                                             if replay_check is not None and args.timed_stage_events
                                             else None),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        td.destroy_process_group()


SWEEP_LOG2 = (14, 16, 18, 20, 22, 24, 26)


def bench_batch_sweep(args, lib, n_keys: int, dev, sizes=SWEEP_LOG2):
    """Config B's key space at batch sizes 2^14 .. 2^26 (the regime of
    the host's micro-batching submitter, SURVEY §8(b) threading), after the timed region.
    Per size a fresh engine (pipeline off, one stream) decides warm-up + timed batches of
    uniform keys; reported: decisions/s over the back-to-back timed batches, the per-batch
    latency (enqueue one batch + synchronise, wall clock, median of 5), both on an engine
    without stage events, and the HIP-event stage times of the same batches on a second
    engine that records them (at small sizes the ~14 events per batch are themselves a
    visible share of its time).  Sparse batches (below R/8 requests per bucket on average,
    R = 2048 keys per bucket: up to 2^23 here) send their sparse buckets to k_fold_sparse,
    one wave each, and take hot-key runs only from 2^20; at 2^24 and 2^26 every bucket takes
    k_fold_wide."""
    from distributedratelimiting.redis_amd import TokenBucketEngine
    out = []
    gen_stream = torch.cuda.current_stream(dev).cuda_stream or None
    for lg in sizes:
        n = 1 << lg
        warm, timed = (3, 10) if lg <= 22 else (2, 5)
        eng = TokenBucketEngine(n_keys, args.token_limit, args.tokens_per_period, args.period_ticks,
                                device=dev.index, stage_timing=False, max_batch=n, pipeline=False)
        sparse = eng.batch_format(n)["sparse"]
        bufs = []
        for s in range(warm + timed + 5):
            k = torch.empty(n, dtype=torch.int64, device=dev)
            p = torch.empty(n, dtype=torch.int32, device=dev)
            t = torch.empty(n, dtype=torch.int64, device=dev)
            assert lib.tbe_gen_batch_device(SEED_B ^ 0x5A, n_keys, s * n, n, 1, 1, T0_US + s * args.interval_us,
                                            args.interval_us, k.data_ptr(), p.data_ptr(), t.data_ptr(),
                                            gen_stream) == 0
            if args.sweep_zipf:
                assert lib.tbe_gen_zipf_keys_device(SEED_B ^ 0x5A, n_keys, args.zipf_s, s * n, n, k.data_ptr(),
                                                    gen_stream) == 0
            bufs.append((k, p, t))
        g = torch.empty(n, dtype=torch.uint8, device=dev)
        r = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        for s in range(warm):
            eng.acquire_batch_device(*bufs[s], g, r)
        eng.synchronize()
        t0 = time.perf_counter()
        for s in range(warm, warm + timed):
            eng.acquire_batch_device(*bufs[s], g, r)
        eng.synchronize()
        elapsed = time.perf_counter() - t0
        lat = []
        for s in range(warm + timed, warm + timed + 5):
            t1 = time.perf_counter()
            eng.acquire_batch_device(*bufs[s], g, r)
            eng.synchronize()
            lat.append(time.perf_counter() - t1)
        eng.close()
        # the same batches on an engine that records stage events
        eng = TokenBucketEngine(n_keys, args.token_limit, args.tokens_per_period, args.period_ticks,
                                device=dev.index, stage_timing=True, max_batch=n, pipeline=False)
        for s in range(warm + timed):
            if s == warm:
                eng.synchronize()
                eng.stage_times()
            eng.acquire_batch_device(*bufs[s], g, r)
        eng.synchronize()
        st = eng.stage_times()
        eng.close()
        del bufs
        out.append({"batch": n, "batches_timed": timed, "ms_per_batch": round(elapsed / timed * 1e3, 4),
                    "decisions_per_s": round(n * timed / elapsed, 1),
                    "latency_ms": round(float(np.median(lat)) * 1e3, 4),
                    "stage_ms_per_batch": {k: round(v / timed, 4) for k, v in st.items()},
                    "fold": ("k_fold_sparse (one wave per sparse bucket) + k_fold_wide (listed dense buckets)"
                             if sparse else "k_fold_wide (every bucket)")})
    torch.cuda.empty_cache()
    return out


def bench_strdir(batches, n_keys: int, dev):
    """Key text "user-<key>" of consecutive config-B batches through the device string
    directory (tbe_sdir_assign_device, automatic path choice), HIP events on the
    directory's stream: batch 0 is cold (every key new); the known share then grows batch
    by batch (1e8 keys, 2^26 requests per batch: ~96% known by the sixth), so the last
    batch is the steady state the warm path serves.  A lookup of the last batch is timed
    too.  The ids must equal the u64 directory's on the same keys (both assign by first
    occurrence), a size-independent check of the string path at full scale."""
    import torch
    from distributedratelimiting.redis_amd import cluster
    from distributedratelimiting.redis_amd.strdir import StringDirectory, synthetic_key_text
    out = {}
    with torch.cuda.stream(torch.cuda.Stream(dev)):
        sd = StringDirectory(n_keys, 16 * n_keys + (1 << 20), prefix="bench:", device=dev.index)
        ud = cluster.DeviceDirectory(n_keys, device=dev.index)
        per, same, known_before, text_bytes = [], True, 0, 0
        look = None
        for j, b in enumerate(batches):
            buf, offs, nb = synthetic_key_text(b[0], "user-")
            text_bytes = nb
            torch.cuda.synchronize(dev)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            ids = sd.assign(buf, offs, nb)
            ev[1].record()
            if j == len(batches) - 1:
                e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e2[0].record()
                lk = sd.lookup(buf, offs, nb)
                e2[1].record()
                torch.cuda.synchronize(dev)
                look = b[0].numel() / (e2[0].elapsed_time(e2[1]) / 1e3)
                same = same and bool(torch.equal(lk, ids))
            same = same and bool(torch.equal(ids, ud.assign(b[0])))
            torch.cuda.synchronize(dev)
            size = sd.size()
            n = b[0].numel()
            per.append({"batch": j, "new_keys": size - known_before, "new_share": round((size - known_before) / n, 4),
                        "assign_per_s": round(n / (ev[0].elapsed_time(ev[1]) / 1e3), 1)})
            known_before = size
            del buf, offs, ids
        n = batches[0][0].numel()
        out = {"batch": n, "key_text_bytes": int(text_bytes),
               "cold_assign_per_s": per[0]["assign_per_s"],
               "warm_assign_per_s": per[-1]["assign_per_s"],
               "warm_new_share": per[-1]["new_share"],
               "lookup_per_s": round(look, 1), "per_batch": per,
               "ids": sd.size(), "ids_equal_u64_directory": same,
               "note": "key text 'user-<config-B key>' (prefix 'bench:'), exact byte compare; cold = batch 0 "
                       "(all keys new), warm = the last of the consecutive batches (steady state; the automatic "
                       "choice takes the warm path once a batch brings < 50% new keys)"}
        sd.close()
        ud.close()
    return out


def algorithmic_bytes(stage: str, n: int, n_keys: int, passes: int, packed: bool,
                      distinct: float = None, reply: int = 4, written: float = None) -> int:
    """Bytes one launch of `stage` must move at minimum for its function,
    averaged over the passes where a stage runs once per pass.  Packed: the passes and
    the fold move one 8-byte record per request; wide: {key u32, permits i32, ts i64}.
    A pass writes each input element's one-byte digit, its inverse reads it (k_unrank)."""
    rec = 8 if packed else 16
    u = distinct if distinct is not None else n_keys * (1.0 - np.exp(-n / n_keys))
    if stage == "fold":
        # sorted records + reply (4 bytes, or 1 when TokenLimit <= 127) per request; the rows
        # of the distinct keys read (16 B) and of the keys modified written (16 B)
        w = written if written is not None else u
        return int(n * (rec + reply) + u * 16 + w * 16)
    if stage == "scatter":
        # pass 0 reads the caller's key 8 + permits 4 + ts 8, later passes one record;
        # every pass writes a record and its input's one-byte digit
        return int(n * ((20 + rec * (passes - 1)) / passes + rec + 1))
    if stage == "hist":
        return int(n * (8 + (8 if packed else 4) * (passes - 1)) / passes)
    if stage == "bounds":
        return n * (8 if packed else 4)
    if stage == "unscatter":
        # digit 1 + gathered reply + written reply (inner passes) or 5 (final: u8 + i32)
        return int(n * ((1 + 2 * reply) * (passes - 1) + 1 + reply + 5) / passes)
    return n * 4


def algorithmic_note(stage: str, layout: dict, u: int, w: int) -> str:
    r = 1 if layout.get("narrow") else 4
    rec = 8 if layout.get("packed") else 16
    if stage == "fold":
        return (f"fold: n*({rec} record + {r} reply) + 16*U rows read + 16*W rows written "
                f"(U={u}, W={w}: per-batch mean over the timed batches when the replay ran)")
    return f"{stage}: DESIGN.md §5 per-launch minimum (bench.algorithmic_bytes)"


PMC_SOURCE = ("profiles/pmc_summary.json: rocprofv3 --pmc passes of tools/pmc_passes.sh over bench.py "
              "--steps 20 --warmup 5, dispatches between the timed-region markers only, bytes by the "
              "calibrated read/write models")


def pmc_stage(w, stage: str):
    """HBM bytes per step of one bench stage (all its kernels' timed launches), from a PMC
    summary entry matched to this run (bench_kinds.pmc_workload), if any."""
    st = (w or {}).get("stages", {}).get(stage)
    return st.get("hbm_bytes_per_step") if st else None


def pmc_step_traffic(w):
    """HBM bytes of one whole step (every kernel of one timed batch), from a matched PMC
    summary entry, if any."""
    return round(w["step_hbm_bytes"], 1) if w and "step_hbm_bytes" in w else None


def workload_name(args, n: int) -> str:
    if args.workload == "testapp":
        return (f"TestApp TokenBucket limiter (TokenLimit {args.token_limit}, {args.tokens_per_period}/s), "
                f"{n}-request batches spanning {args.interval_us / 1e6:g} s each (config A)")
    if args.workload == "zipf":
        return (f"TokenBucket Zipf({args.zipf_s}) over each GPU's keys, 2^{n.bit_length() - 1}-request "
                "batches (config C per-GPU slice)")
    return f"TokenBucket uniform keys, 2^{n.bit_length() - 1}-request batches (config B)"


def cpu_baseline(args, n_keys: int, zkeys=(), seed_b: int = SEED_B):
    """The C restatement of the reference script (oracle/tb_ref.c, serial like Redis'
    single script thread) timed on the same trace: the first `sample` requests of each
    batch, batches in order, until ~args.cpu_seconds of CPU work.  Beside it, the same
    restatement key-sharded over CPU_THREADS host threads (SURVEY.md §8d "all host
    cores"; 16 = the GPU box's CPU share), on a fresh table and a shorter sample."""
    from oracle import cref  # CPU baseline leg (checker library), never the product path
    from distributedratelimiting.redis_amd import fill_rate

    sample = min(args.batch, 1 << 22)
    seed = SEED_C if zkeys else seed_b

    def timed(threads: int, seconds: float):
        ref = cref.CTokenBucket(n_keys, args.token_limit, fill_rate(args.tokens_per_period, args.period_ticks))
        done, spent, b = 0, 0.0, 0
        while spent < seconds and b < 64:
            k, p, t = cref.gen_batch(seed, n_keys, b, args.batch, args.interval_us)
            if zkeys:
                k = zkeys[b % len(zkeys)]
            k, p, t = k[:sample], p[:sample], t[:sample]
            t0 = time.perf_counter()
            ref.acquire_batch(k, p, t, threads=threads)
            spent += time.perf_counter() - t0
            done += sample
            b += 1
        ref.close()
        return done, spent, b

    done, spent, b = timed(1, args.cpu_seconds)
    what = "config-C (Zipf)" if zkeys else ("config-A (TestApp)" if seed_b == SEED_A else "config-B")
    out = {"value": round(done / spent, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
           "sample": f"first {sample} requests of each of {b} {what} batches "
                     f"({done} decisions, {spent:.1f} s), oracle/tb_ref.c single thread",
           "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}
    if CPU_THREADS > 1 and args.cpu_seconds > 0:
        done_t, spent_t, b_t = timed(CPU_THREADS, min(args.cpu_seconds, 4.0))
        out["sharded"] = {"value": round(done_t / spent_t, 1), "unit": "decisions/s", "cores": CPU_THREADS,
                          "kind": "port",
                          "sample": f"first {sample} requests of each of {b_t} {what} batches "
                                    f"({done_t} decisions, {spent_t:.1f} s), oracle/tb_ref.c "
                                    f"key-sharded (key % {CPU_THREADS}) over {CPU_THREADS} threads",
                          "cores_note": f"{CPU_THREADS} = the host-CPU share a one-GPU job gets on the GPU box "
                                        f"(os.cpu_count() reports the whole machine, {os.cpu_count()})"}
    return out


CPU_THREADS = 16
REHEARSAL_NOTE = ("--share-device: every rank on cuda:0 over gloo (collectives staged through host "
                  "memory); exercises the multi-rank path, times are not a scaling measurement")


if __name__ == "__main__":
    main()
