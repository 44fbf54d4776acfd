"""bench.py --workload queue | approx: SURVEY.md §8d configs D and E.

Config D (TokenBucketWithQueue, Q): 1e8 keys (ceil(1e8 / N) per rank), 2^26-request
batches, permits 1, TokenLimit 4, 1 token / s, QueueLimit 16, OldestFirst, 1 ms of
injected time per batch (demand >> fill, so queues saturate).  A step is one
WaitAsyncCore batch (tbe_wait_batch_device) plus the replenish tick at the batch's end
(tbe_refresh_device, Q:237-271), both on device buffers.

Config E (ApproximateTokenBucket, A): 1e7 shared keys replicated on every rank, each rank
decides its own 2^26 AcquireCore requests per batch over them, then one refresh epoch:
collect the local counts (A:430-435), exchange them between the ranks (RCCL all-gather
over xGMI; nothing to exchange at N = 1), and replay the sync script for every client in
rank order with staggered timestamps T + r*P/N (A:241-270, SURVEY.md §8e option 2).

value = all ranks' requests / max-over-ranks time (weak scaling); per-stage times come
from the engine's HIP events, the refresh kernels' from HIP events on the same stream.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

HBM_PEAK_GBS = 8000.0
SEED_D = 0x5EED000D
SEED_E = 0x5EED000E
T0_US = 1_760_000_000_000_000
METRIC = "acquire decisions/sec (node) at 100M keys, 1/2/4/8 GPU; % HBM roofline"


def _gen(lib, seed, n_keys, s, n, interval_us, dev):
    k = torch.empty(n, dtype=torch.int64, device=dev)
    p = torch.empty(n, dtype=torch.int32, device=dev)
    t = torch.empty(n, dtype=torch.int64, device=dev)
    rc = lib.tbe_gen_batch_device(seed, n_keys, s * n, n, 1, 1, T0_US + s * interval_us, interval_us,
                                  k.data_ptr(), p.data_ptr(), t.data_ptr(), None)
    assert rc == 0
    return k, p, t


def cpu_model() -> str:
    """The host CPU's model name (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _distinct(n: int, k: int) -> float:
    return k * (1.0 - np.exp(-n / k))


PMC_SUMMARY = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_summary.json")
# what makes two runs move the same bytes per step: the fingerprint of a bench run, written
# by the PMC passes' own bench runs (tools/pmc_passes.sh sets TBE_PMC_FINGERPRINT) into
# profiles/pmc_summary.json and compared key by key with the run that reports the bytes
FINGERPRINT_KEYS = ("workload", "world", "keys_per_gpu", "batch", "steps", "warmup", "token_limit",
                    "tokens_per_period", "period_ticks", "interval_us", "queue_limit", "route",
                    "owner_map", "share_device", "layout", "engine_sources_sha256")


def run_fingerprint(args, world: int, keys_per_gpu: int, layout: dict) -> dict:
    """The fingerprint of this bench run (FINGERPRINT_KEYS); the engine's sources by the
    same SHA-256 the build stamps beside libtbe.so (sources + compiler flags)."""
    from distributedratelimiting.redis_amd.build import DEPS, HIPCC_FLAGS, _digest
    return {"workload": args.workload, "world": int(world), "keys_per_gpu": int(keys_per_gpu),
            "batch": int(args.batch), "steps": int(args.steps), "warmup": int(args.warmup),
            "token_limit": int(args.token_limit), "tokens_per_period": int(args.tokens_per_period),
            "period_ticks": int(args.period_ticks), "interval_us": int(args.interval_us),
            "queue_limit": int(args.queue_limit) if args.workload == "queue" else None,
            "route": args.route if world > 1 else None,
            "owner_map": getattr(args, "owner_map", None) if world > 1 else None,
            "share_device": bool(args.share_device),
            "layout": {k: layout[k] for k in sorted(layout)},
            "engine_sources_sha256": _digest(DEPS, HIPCC_FLAGS)}


def write_fingerprint(fp: dict) -> None:
    """bench runs under tools/pmc_passes.sh record what they ran (TBE_PMC_FINGERPRINT)."""
    import json
    path = os.environ.get("TBE_PMC_FINGERPRINT")
    if path:
        with open(path, "w") as f:
            json.dump(fp, f, indent=1, sort_keys=True)


def pmc_workload(workload: str, fp: dict, path: str = PMC_SUMMARY):
    """(the PMC summary's entry for `workload`, None) when it was measured on a run with
    exactly this fingerprint, else (None, reason).  A run whose configuration differs
    (keys per GPU, batch, world, schedule, layout, engine sources...) gets no bytes."""
    import json
    try:
        with open(path) as f:
            w = json.load(f).get("workloads", {}).get(workload)
    except (OSError, ValueError) as e:
        return None, f"no PMC summary ({type(e).__name__})"
    if w is None:
        return None, f"no PMC passes for workload {workload!r}"
    got = w.get("fingerprint")
    if got is None:
        return None, "the PMC passes recorded no run fingerprint"
    diff = [k for k in FINGERPRINT_KEYS if got.get(k) != fp.get(k)]
    if diff:
        return None, "PMC passes ran a different configuration: " + ", ".join(
            f"{k} {got.get(k)!r} != {fp.get(k)!r}" if k != "layout" else "layout" for k in diff)
    return w, None


def _pmc_traffic(w, kernels):
    """HBM bytes per launch of the named kernels (mean over them) in a matched PMC entry."""
    if w is None:
        return None
    d = w.get("kernels", {})

    def entry(k):   # "k_fold_q<true>" also names k_fold_q<true, HW> (any queue-header width)
        if k in d:
            return d[k]
        m = [d[x] for x in d if k.endswith(">") and x.startswith(k[:-1] + ",")]
        return m[0] if len(m) == 1 else {}
    v = [entry(k)["hbm_bytes_per_launch"] for k in kernels if "hbm_bytes_per_launch" in entry(k)]
    return round(sum(v) / len(v), 1) if len(v) == len(kernels) and v else None


PMC_KERNELS = {
    ("queue", "fold"): ["k_fold_q<true>"],
    ("queue", "drain"): ["k_drain"],
    ("queue", "scatter"): ["k_scatter_rec<true, false, true, false>", "k_scatter_rec<false, false, true, false>"],
    ("approx", "fold"): ["k_fold_a<true>"],
    ("approx", "scatter"): ["k_scatter_rec<true, false, false, true>", "k_scatter_rec<false, false, false, false>"],
}


def _roofline(fold_ms, step_alg, step_note, own_alg, own_note, workload, fp, ms_per_step, stages, steps,
              pmc_key=None):
    """SURVEY.md §8(d) roofline of one bench line: the decision kernel
    (the fold) is the dominant kernel; `achieved` = the step's algorithmic bytes B_alg over
    the fold's average launch time, `frac` = achieved / 8 TB/s.  The fold's own byte count
    is kept as kernel_own_*; step_* relate B_alg to the whole timed step; `traffic` and
    `step_traffic` are the PMC bytes (tools/pmc_summary.py) of a run with exactly this
    fingerprint, else null with the reason."""
    if not fold_ms > 0:    # --no-stage-timing: no kernel times
        return None
    achieved = step_alg / (fold_ms * 1e-3) / 1e9
    step_achieved = step_alg / (ms_per_step * 1e-3) / 1e9
    key = pmc_key or workload
    w, why = pmc_workload(key, fp)
    traffic = _pmc_traffic(w, PMC_KERNELS[(workload, "fold")]) if (workload, "fold") in PMC_KERNELS else None
    if w is not None and traffic is None:
        why = "no PMC bytes for the fold kernels"
    st = w.get("step_hbm_bytes") if w is not None else None
    largest = max(stages, key=stages.get) if stages else None
    return {"bound": "hbm", "kernel": "fold", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            **({"traffic_null_reason": why} if traffic is None else {}),
            "alg_bytes_per_launch": int(step_alg), "alg_bytes_note": "SURVEY.md §8(d) B_alg of the step: " + step_note,
            "avg_launch_ms": round(fold_ms, 4),
            "kernel_own_bytes": int(own_alg), "kernel_own_note": own_note,
            "kernel_own_frac": round(own_alg / (fold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            **({"largest_stage": largest, "largest_stage_ms_per_step": round(stages[largest] / steps, 4)}
               if largest else {}),
            "step_alg_bytes": int(step_alg), "step_achieved": round(step_achieved, 1),
            "step_frac": round(step_achieved / HBM_PEAK_GBS, 4),
            "step_traffic": round(st, 1) if st is not None else None,
            **({"step_traffic_null_reason": why or "no step bytes in the PMC summary"} if st is None else {}),
            "timing": "HIP events around the fold on the engine's launch stream over the timed region",
            "fingerprint": fp}


def run(args, lib, dev, world, rank, dist):
    if args.workload == "queue":
        return run_queue(args, lib, dev, world, rank, dist)
    return run_approx(args, lib, dev, world, rank, dist)


def reduce_max(x: float, dev) -> float:
    """Max over ranks of a host scalar (RCCL on the device; gloo on the host)."""
    import torch.distributed as td
    t = torch.tensor([x], dtype=torch.float64, device=dev if td.get_backend() != "gloo" else "cpu")
    td.all_reduce(t, op=td.ReduceOp.MAX)
    return float(t.item())


def gather_floats(x: float, world: int, dev):
    """Every rank's host scalar, in rank order."""
    import torch.distributed as td
    d = dev if td.get_backend() != "gloo" else "cpu"
    mine = torch.tensor([x], dtype=torch.float64, device=d)
    every = torch.empty(world, dtype=torch.float64, device=d)
    td.all_gather_into_tensor(every, mine)
    return every.cpu().numpy()



_MARK_STREAM = {}


def mark(lib, tag: int, dev) -> None:
    """k_mark<tag> dispatch (include/tbe_tools.h): tools/pmc_summary.py keeps the
    dispatches enqueued between marker 1 and marker 2, i.e. exactly the timed batches.
    On a stream of its own, outside the timed region."""
    import ctypes
    if dev not in _MARK_STREAM:
        lib.tbe_mark_device.restype = ctypes.c_int
        lib.tbe_mark_device.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
        _MARK_STREAM[dev] = torch.cuda.Stream(dev)
    # a profiling aid only: a library without this marker (an older A/B build) just skips it
    lib.tbe_mark_device(tag, _MARK_STREAM[dev].cuda_stream)


def _barrier_time(dist, dev, t0):
    torch.cuda.synchronize()
    if dist:
        import torch.distributed as td
        td.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        elapsed = reduce_max(elapsed, dev)
    return elapsed


def _queue_pass(args, lib, dev, world, dist, kl, period_ticks, seed, marked=False):
    """One config-D schedule (warm-up + timed batches, each with its tick) on a fresh
    engine; returns the timing, stage times and outcome counts."""
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine

    n, steps, warm = args.batch, args.steps, args.warmup
    total = warm + steps

    def new_engine(timing):
        return QueueingTokenBucketEngine(kl, args.token_limit, args.tokens_per_period, period_ticks,
                                         args.queue_limit, 0, device=dev.index, stage_timing=timing,
                                         max_batch=n, pack=not args.no_pack, fold_records=not args.unscatter_all,
                                         digit_stream=not args.hist_records, rerank=args.rerank)

    # the timed engine records events around the fold alone (the roofline's kernel time, two
    # events per batch: a pair per stage would leave the stream idle ~14 times a batch); the
    # stage breakdown comes from a replay of the same schedule afterwards
    # inputs first, then the engine -- the order bench.py uses for configs B and C (an engine
    # created before 33 GB of inputs ran its fold 20-25% slower than the same engine created
    # after them: profiles/r06h_settle_ab.log, r06i_*; CHANGELOG round 6)
    timing = False if args.no_stage_timing else True if args.timed_stage_events else "fold"
    eng = new_engine(timing) if args.engine_first else None   # (A/B: round 5's order)
    bufs = [_gen(lib, seed, kl, s, n, args.interval_us, dev) for s in range(total)]
    torch.cuda.synchronize()
    if eng is None:
        eng = new_engine(timing)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    rem = torch.empty(n, dtype=torch.int32, device=dev)
    # drain log: a tick grants at most min(QueueLimit, TokenLimit) entries per key
    cap = min(kl * min(max(1, args.queue_limit), args.token_limit), total * n)
    lk = torch.empty(cap, dtype=torch.int64, device=dev)
    li = torch.empty(cap, dtype=torch.int64, device=dev)
    lr = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(total, dtype=torch.int32, device=dev)   # one drain count per tick
    queued = torch.zeros(total, dtype=torch.int64, device=dev)
    # a stream of our own (the default stream's handle is NULL, which the engine reads as
    # "its own stream"), so the drain's HIP events sit on the stream the kernels run on
    stream = torch.cuda.Stream(dev)
    sh = stream.cuda_stream
    torch.cuda.synchronize()
    fused = not args.no_fuse_tick

    def step(s, ev=None):
        tick = T0_US + (s + 1) * args.interval_us
        c = cnt[s:s + 1]
        if fused:   # the tick drains inside the batch's fold (tbe_wait_batch_tick_device)
            eng.wait_batch_tick_device(*bufs[s], st, rem, s * n, tick, lk, li, lr, c, stream=sh)
            return
        eng.wait_batch_device(*bufs[s], st, rem, id_base=s * n, stream=sh)
        if ev:
            ev[0].record(stream)
        eng.refresh_device(tick, lk, li, lr, c, stream=sh)
        if ev:
            ev[1].record(stream)

    def outcome(s):   # enqueues of batch s (outside the timed region: warm-up only)
        with torch.cuda.stream(stream):
            queued[s] = (st == 2).sum()

    for s in range(warm):
        step(s)
        outcome(s)
    torch.cuda.synchronize()
    eng.synchronize()
    eng.stage_times()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    if marked:
        mark(lib, 1, dev)
    if dist:
        import torch.distributed as td
        td.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, s in enumerate(range(warm, total)):
        step(s, evs[i])
    elapsed = _barrier_time(dist, dev, t0)
    if marked:
        mark(lib, 2, dev)
    eng.synchronize()
    stages = eng.stage_times()
    fold_timed = stages.get("fold", 0.0)
    drain_ms = 0.0 if fused else sum(a.elapsed_time(b) for a, b in evs)
    outcome(total - 1)
    torch.cuda.synchronize()
    grants = cnt.cpu().numpy().astype(np.int64)
    q = queued.cpu().numpy()
    granted = float((st == 1).float().mean().item())
    layout = eng.layout()
    if not args.no_stage_timing and not args.timed_stage_events:
        # the replay: a fresh engine with stage events decides the same schedule (same state
        # batch by batch); its replies are the timed run's
        g_timed, r_timed = st.clone(), rem.clone()
        eng.close()
        eng = new_engine(True)
        cnt.zero_()
        for s in range(warm):
            step(s)
        eng.synchronize()
        eng.stage_times()
        for s in range(warm, total):
            step(s)
        eng.synchronize()
        stages = eng.stage_times()
        torch.cuda.synchronize()
        assert torch.equal(st, g_timed) and torch.equal(rem, r_timed), "stage replay diverged from the timed run"
    if not fused:
        stages["drain"] = drain_ms
    out = {"elapsed": elapsed, "stages": stages, "granted": granted, "q_last": int(q[-1]),
           "tick_grants_per_step": grants[warm:].tolist(), "d_last": int(grants[-1]),
           "queued_warmup": q[:warm].tolist(), "layout": layout, "fold_timed": fold_timed}
    eng.close()
    return out


def run_queue(args, lib, dev, world, rank, dist):
    keys_total = args.keys or 100_000_000
    kl = (keys_total + world - 1) // world
    n, steps = args.batch, args.steps
    seed = SEED_D + 7919 * rank
    fused = not args.no_fuse_tick
    # the PMC markers go around the headline schedule's timed batches, or with --drain-marked
    # around the draining schedule's (tools/pmc_passes.sh's "queue_draining" run)
    r = _queue_pass(args, lib, dev, world, dist, kl, args.period_ticks, seed, marked=not args.drain_marked)
    elapsed, stages, granted, q_last, d_last = r["elapsed"], r["stages"], r["granted"], r["q_last"], r["d_last"]
    fp = run_fingerprint(args, world, kl, r["layout"])
    if rank == 0 and not args.drain_marked:
        write_fingerprint(fp)

    value = n * steps * world / elapsed
    u = _distinct(n, kl)
    packed = bool(r["layout"].get("packed"))
    # the fold's own bytes: records (packed: u64 record 8 + arrival index 4; wide: key 4,
    # permits 4, ts 8, index 4) + packed reply 4 per request; per distinct key: bucket row
    # 16 + queue header (4 bytes at QueueLimit <= 1024, else 8), read and written; 8 per enqueue
    rec = 12 if packed else 20
    per_u = 2 * (16 + (4 if r["layout"].get("queue_header_32") else 8))
    own = n * (rec + 4) + u * per_u + q_last * 8
    own_note = f"fold: n*{rec + 4} + distinct*{per_u} + enqueued*8 (last batch's enqueues)"
    # the B formula (W ~ distinct keys x grant share) + 8 B per
    # enqueue + 8 B per dequeue (lower bound: headers of non-empty queues omitted)
    step_alg = n * 25 + u * 16 + u * granted * 16 + q_last * 8 + d_last * 8
    step_note = "25*N + 16*U + 16*U*granted_frac + 8*enqueued + 8*dequeued (last batch)"
    fold_ms = (r["fold_timed"] if r["fold_timed"] > 0 else stages.get("fold", 0.0)) / steps
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "decisions/s", "n_gpus": world,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (splitmix64 seeded trace generated in HBM)",
        "config": {"workload": f"TokenBucketWithQueue OldestFirst, QueueLimit {args.queue_limit}, "
                               f"2^{n.bit_length() - 1}-request batches + replenish tick (config D)",
                   "keys_total": keys_total, "keys_per_gpu": kl, "batch_per_gpu": n,
                   "token_limit": args.token_limit, "tokens_per_period": args.tokens_per_period,
                   "period_ticks": args.period_ticks, "interval_us": args.interval_us,
                   "partitioning": f"key-hash x{world}, no data-path collective",
                   "tick": "fused into the batch's fold (tbe_wait_batch_tick_device)" if fused
                   else "own pass (tbe_refresh_device)"},
        "last_batch": {"granted_frac": round(granted, 4), "queued": q_last, "tick_grants": d_last},
        "tick_grants_per_step": r["tick_grants_per_step"],
        "stage_ms_per_step": {k: round(v / steps, 4) for k, v in stages.items()},
        "roofline": _roofline(fold_ms, step_alg, step_note, own, own_note, "queue", fp,
                              elapsed / steps * 1e3, stages, steps),
        "cpu_baseline": None,
    }
    if not args.no_drain_variant:
        # The same schedule with ticks that grant: at 1 token/s a saturated key frees one
        # queue entry per ~1000 ticks, so config D's ticks drain nothing within a run.  With
        # ReplenishmentPeriod = 2 batch intervals every queued key gains half a token per
        # tick, and the FIFO drain (Q:237-271) completes millions of entries per tick.
        pt = 2 * args.interval_us * 10
        d = _queue_pass(args, lib, dev, world, dist, kl, pt, seed, marked=args.drain_marked)
        g = np.array(d["tick_grants_per_step"], dtype=np.float64)
        # the draining schedule's roofline, by the same rule (its PMC bytes come from
        # tools/pmc_passes.sh's "queue_draining" run: --drain-marked puts the markers here)
        dfp = run_fingerprint(args, world, kl, d["layout"])
        dfp["period_ticks"] = pt
        dfp["schedule"] = "draining"
        if rank == 0 and args.drain_marked:
            write_fingerprint(dfp)
        d_step = n * 25 + u * 16 + u * d["granted"] * 16 + d["q_last"] * 8 + d["d_last"] * 8
        d_own = n * (rec + 4) + u * per_u + d["q_last"] * 8 + d["d_last"] * 28
        d_fold = (d["fold_timed"] if d["fold_timed"] > 0 else d["stages"].get("fold", 0.0)) / steps
        line["draining"] = {
            "period_ticks": pt, "tokens_per_period": args.tokens_per_period,
            "value": round(n * steps * world / d["elapsed"], 1),
            "ms_per_step": round(d["elapsed"] / steps * 1e3, 4),
            "tick_grants_per_step": d["tick_grants_per_step"],
            "tick_grants_mean": round(float(g.mean()), 1) if g.size else 0.0,
            "granted_frac_last_batch": round(d["granted"], 4), "queued_last_batch": d["q_last"],
            "stage_ms_per_step": {k: round(v / steps, 4) for k, v in d["stages"].items()},
            "roofline": _roofline(d_fold, d_step, step_note, d_own, own_note + " + dequeued*28 (ring entry + log)",
                                  "queue", dfp, d["elapsed"] / steps * 1e3, d["stages"], steps,
                                  pmc_key="queue_draining"),
            "note": "config D's schedule with ReplenishmentPeriod = 2 batch intervals: the fused ticks "
                    "drain queued entries every step (tick_grants = entries completed by each timed tick)"}
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_queue(args, kl)
    return line


def cpu_queue(args, kl):
    """oracle/tb_ref.c tbrq_* (serial): the first 2^20 requests of each config-D batch,
    each followed by that batch's tick, until ~args.cpu_seconds."""
    from oracle import cref
    from distributedratelimiting.redis_amd import fill_rate

    ref = cref.CQueueingTokenBucket(kl, args.token_limit, fill_rate(args.tokens_per_period, args.period_ticks),
                                    args.queue_limit, 0)
    sample = min(args.batch, 1 << 20)
    done, spent, b = 0, 0.0, 0
    while spent < args.cpu_seconds and b < 64:
        k, p, t = cref.gen_batch(SEED_D, kl, b, args.batch, args.interval_us)
        k, p, t = k[:sample], p[:sample], t[:sample]
        t0 = time.perf_counter()
        ref.acquire_batch(k, p, t, b * args.batch)
        ref.refresh(T0_US + (b + 1) * args.interval_us)
        spent += time.perf_counter() - t0
        done += sample
        b += 1
    ref.close()
    return {"value": round(done / spent, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} requests of each of {b} config-D batches + their ticks "
                      f"({done} decisions, {spent:.1f} s), oracle/tb_ref.c tbrq_* single thread",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}


def run_approx(args, lib, dev, world, rank, dist):
    from distributedratelimiting.redis_amd import ApproximateEngine

    kshared = args.keys or 10_000_000
    n, steps, warm = args.batch, args.steps, args.warmup
    total = warm + steps
    def new_engine(timing):
        return ApproximateEngine(kshared, args.token_limit, args.tokens_per_period, args.period_ticks,
                                 0, 0, device=dev.index, stage_timing=timing, max_batch=n,
                                 pack=not args.no_pack, fold_records=not args.unscatter_all,
                                 digit_stream=not args.hist_records, rerank=args.rerank)

    # fold events alone in the timed engine; the stage breakdown comes from a replay (below).
    # Inputs first, then the engine, as for configs B, C and D
    seed = SEED_E + 7919 * rank
    bufs = [_gen(lib, seed, kshared, s, n, args.interval_us, dev)[:2] for s in range(total)]
    torch.cuda.synchronize()
    eng = new_engine(False if args.no_stage_timing else True if args.timed_stage_events else "fold")
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    av = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.empty(kshared, dtype=torch.int32, device=dev)
    allc = torch.empty(kshared * world, dtype=torch.int32, device=dev) if dist else counts
    period_us = args.period_ticks // 10
    stagger = period_us // world
    torch.cuda.synchronize()
    refresh_s = {"node": [0.0, 0], "clients": [0.0, 0]}
    from distributedratelimiting.redis_amd import cluster

    def refresh(s, mode, timed):
        t1 = time.perf_counter()
        ts = T0_US + (s + 1) * args.interval_us
        if mode == "node" and not dist:
            # one client, nothing to exchange: RefreshAsync as one engine call (A:412-508)
            eng.refresh(ts)
            if timed:
                refresh_s[mode][0] += time.perf_counter() - t1
                refresh_s[mode][1] += 1
            return
        eng.collect(counts)             # A:430-435
        if mode == "node":
            if dist:                    # RCCL all-reduce over xGMI: the node is ONE client
                cluster._all_reduce_sum(counts)
                torch.cuda.current_stream(dev).synchronize()
            eng.sync(counts, 1, 0, ts, 0)
        else:
            if dist:                    # RCCL all-gather: every rank a client
                cluster._all_gather(allc, counts)
                torch.cuda.current_stream(dev).synchronize()   # the sync replay reads allc
            eng.sync(allc, world, rank, ts, stagger)
        if timed:
            refresh_s[mode][0] += time.perf_counter() - t1
            refresh_s[mode][1] += 1

    def step(s, timed=False):
        # everything on the engine's stream; collect synchronises it
        eng.acquire_batch_device(*bufs[s], st, av, wait=False, id_base=s * n)
        if timed:   # collect would wait for the batch anyway; this keeps it out of refresh time
            torch.cuda.synchronize()
        refresh(s, args.approx_mode, timed)

    for s in range(warm):
        step(s)
    torch.cuda.synchronize()
    eng.synchronize()
    eng.stage_times()
    mark(lib, 1, dev)
    if dist:
        import torch.distributed as td
        td.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(warm, total):
        step(s, timed=True)
    elapsed = _barrier_time(dist, dev, t0)
    mark(lib, 2, dev)
    eng.synchronize()
    stages = eng.stage_times()
    fold_timed = stages.get("fold", 0.0)
    granted = float((st == 1).float().mean().item())
    # the other exchange mode's refresh epoch, timed after the timed region on the same
    # engine (its counts are the last batch's local scores, then zeros)
    alt = "clients" if args.approx_mode == "node" else "node"
    if dist:
        td.barrier()
    for j in range(min(steps, 5)):
        refresh(total + j, alt, True)
    refresh_ms = {m: round(v[0] / v[1] * 1e3, 4) if v[1] else None for m, v in refresh_s.items()}
    if dist:
        refresh_ms = {m: round(reduce_max(v, dev), 4) if v is not None else None for m, v in refresh_ms.items()}
    # config E's 8-GPU refresh on this one GPU: the all-gather layout of
    # 8 clients' counts -- 8 consecutive batches' collected local scores stand in for the 8
    # ranks' -- and the client-ordered replay of 8 sync calls per key with staggered times
    eight = approx_eight_clients(args, eng, bufs, st, av, kshared, n, total + 5, dev) if not dist else None
    # bytes each GPU receives per refresh: ring all-reduce 2 (N-1)/N * 4K, all-gather (N-1) * 4K
    xbytes = {"node": int(2 * (world - 1) * kshared * 4 // world), "clients": int((world - 1) * kshared * 4)}
    layout = eng.layout()
    if not args.no_stage_timing and not args.timed_stage_events:
        # stage times from a replay of the warm-up + timed schedule on an engine that records
        # them (the refresh epochs included, as in the timed steps)
        eng.close()
        eng = new_engine(True)
        for s in range(warm):
            step(s)
        eng.synchronize()
        eng.stage_times()
        for s in range(warm, total):
            step(s)
        eng.synchronize()
        stages = eng.stage_times()

    value = n * steps * world / elapsed
    fp = run_fingerprint(args, world, kshared, layout)
    if rank == 0:
        write_fingerprint(fp)
    u = _distinct(n, kshared)
    # the fold's own bytes: records (key 4, permits 4, arrival index 4) + reply 4 per
    # request; local-tier row 16 B read + written per distinct key
    own, own_note = n * 16 + u * 32, "fold: n*16 + distinct*32"
    fold_ms = (fold_timed if fold_timed > 0 else stages.get("fold", 0.0)) / steps
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "decisions/s", "n_gpus": world,
        "steps": steps, "warmup": warm, "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (splitmix64 seeded trace generated in HBM)",
        "config": {"workload": f"ApproximateTokenBucket AcquireCore, {kshared} shared keys, "
                               f"2^{n.bit_length() - 1}-request batches + one refresh epoch per batch "
                               f"(config E)",
                   "keys_shared": kshared, "batch_per_gpu": n, "token_limit": args.token_limit,
                   "tokens_per_period": args.tokens_per_period, "period_ticks": args.period_ticks,
                   "interval_us": args.interval_us, "clients": world,
                   "approx_mode": args.approx_mode,
                   "exchange": ("none (one client)" if not dist else
                                "RCCL all-reduce of int32 counts (the node is one client, SURVEY.md §8e option 1)"
                                if args.approx_mode == "node" else
                                "RCCL all-gather of int32 counts (every rank a client, §8e option 2)")},
        "granted_frac_last_batch": round(granted, 4),
        "stage_ms_per_step": {k: round(v / steps, 4) for k, v in stages.items()},
        "refresh_ms_per_step_wall": refresh_ms[args.approx_mode],
        "refresh_modes": {m: {"ms_per_epoch_wall": refresh_ms[m], "exchange_bytes_per_gpu": xbytes[m],
                              "timed": "in the timed steps" if m == args.approx_mode else
                                       f"{min(steps, 5)} epochs after the timed region"}
                          for m in ("node", "clients")},
        # 8+4+1 in/out + 8 local-tier state per decision,
        # K_shared * (4 count + 24 v,p,t) per refresh
        "roofline": _roofline(fold_ms, n * 21 + kshared * 28, "21*N + 28*K_shared (one refresh per batch)",
                              own, own_note, "approx", fp, elapsed / steps * 1e3, stages, steps),
        **({"eight_client_refresh": eight} if eight is not None else {}),
        "cpu_baseline": None,
    }
    eng.close()
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_approx(args, kshared)
    return line


def approx_eight_clients(args, eng, bufs, st, av, kshared, n, s0, dev, clients: int = 8, epochs: int = 5):
    """The refresh epoch an 8-GPU node runs in config E's clients mode (§8e option 2), on one
    GPU: the counts of `clients` consecutive batches of this engine (each collected after its
    batch: one client's local scores) laid out as RCCL's all-gather lays them out, then
    tbe_approx_sync with n_clients = 8 -- every key's sync script replayed 8 times in client
    order at T + r * P/8 (A:241-270) on this rank's replica.  Wall time per epoch (one engine
    call, synchronous) and the kernel's algorithmic bytes: per key 4 B per client count +
    local tier and client view read/written (16 + 16) + the global tier v, p, t read and
    written (48) = 80 + 4N B, over the bytes the one-client fused refresh moves."""
    allc = torch.empty(clients * kshared, dtype=torch.int32, device=dev)
    for r in range(clients):
        k, p = bufs[r % len(bufs)]
        eng.acquire_batch_device(k, p, st, av, wait=False, id_base=(s0 + r) * n)
        eng.collect(allc[r * kshared:(r + 1) * kshared])
    torch.cuda.synchronize()
    period_us = args.period_ticks // 10
    stagger = period_us // clients
    wall = []
    for j in range(epochs):
        ts = T0_US + (s0 + clients + j) * args.interval_us
        t1 = time.perf_counter()
        eng.sync(allc, clients, 0, ts, stagger)
        wall.append(time.perf_counter() - t1)
    ms = float(np.median(wall)) * 1e3
    alg = kshared * (80 + 4 * clients)
    return {"clients": clients, "epochs_timed": epochs, "ms_per_epoch_wall": round(ms, 4),
            "alg_bytes": alg, "alg_note": f"K_shared * (80 + 4 * {clients}) B",
            "achieved_GBs_wall": round(alg / (ms * 1e-3) / 1e9, 1),
            "counts": f"{clients} consecutive config-E batches' collected local scores, all-gather layout",
            "stagger_us": stagger}


def cpu_approx(args, kshared):
    """oracle/tb_ref.c tba_* (the C restatement of A's local tier and sync, one client, one
    thread): AcquireCore over the first 2^24 requests of each config-E batch, then that
    batch's refresh epoch over every shared key (collect + sync script replay), until
    ~args.cpu_seconds."""
    from oracle import cref

    c = cref.CApprox(kshared, args.token_limit, args.tokens_per_period, args.period_ticks, 0, 0)
    sample = min(args.batch, 1 << 24)
    done, spent, b = 0, 0.0, 0
    while spent < args.cpu_seconds and b < 64:
        k, p, _ = cref.gen_batch(SEED_E, kshared, b, args.batch, args.interval_us)
        k, p = k[:sample], p[:sample]
        t0 = time.perf_counter()
        c.acquire_batch(k, p, wait=False, id_base=b * args.batch, threads=1)
        counts = c.collect()
        c.sync(counts, 1, 0, T0_US + (b + 1) * args.interval_us, 0, threads=1)
        spent += time.perf_counter() - t0
        done += sample
        b += 1
    c.close()
    return {"value": round(done / spent, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} requests of each of {b} config-E batches, each followed by a "
                      f"refresh epoch over all {kshared} keys ({done} decisions, {spent:.1f} s), "
                      f"oracle/tb_ref.c tba_* single thread",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}
