"""bench.py --workload zipf --emulate-world W: config C's ranks at W GPUs, one at a time,
on this one GPU.

Config C is one global Zipf(1.1) stream over 1.25e8 * W keys, W * 2^26 requests per step,
hash-sharded to W owners; the slowest owner sets the node's time
(bench.py takes the max over ranks).  Under the hash partition the hottest key's owner
receives ~1.75x the mean load (SURVEY.md §7 hard part iii).  This leg generates the whole
global stream of every step on the device (the generators bench.py's ranks use, same draw
order), derives every owner's load per step from per-virtual-node counts (exact, for any
owner map), and then runs chosen owners' received streams -- the concatenation over
source ranks of each source's requests for that owner, in arrival order, exactly what
cluster.route_requests delivers -- through a fresh engine on the driver's warm-up + timed
schedule, each behind its own owner key directory.  It does so for two owner maps:
  hash      owner = mix64(key) >> (64 - log2 W), the §8(e) partition;
  balanced  cluster.balanced_owner_map of step 0's virtual-node loads (the mitigation,
            DESIGN.md §7 "owner maps").
The node rate it implies is W * 2^26 / (the slowest emulated owner's ms per step); the
line is marked as an emulation: no other rank shares the chip, and no collective runs.
"""
from __future__ import annotations

import time

import numpy as np
import torch

SEED_C = 0x5EED000C
T0_US = 1_760_000_000_000_000


def _gen(lib, seed, keys_total, s_, g0, n, interval_us, zipf_s, dev, stream, keys_only=False):
    k = torch.empty(n, dtype=torch.int64, device=dev)
    if keys_only:
        assert lib.tbe_gen_zipf_keys_device(seed, keys_total, zipf_s, g0, n, k.data_ptr(), stream) == 0
        return k
    p = torch.empty(n, dtype=torch.int32, device=dev)
    t = torch.empty(n, dtype=torch.int64, device=dev)
    assert lib.tbe_gen_batch_device(seed, keys_total, g0, n, 1, 1, T0_US + s_ * interval_us, interval_us,
                                    k.data_ptr(), p.data_ptr(), t.data_ptr(), stream) == 0
    assert lib.tbe_gen_zipf_keys_device(seed, keys_total, zipf_s, g0, n, k.data_ptr(), stream) == 0
    return k, p, t


def owner_stream(lib, args, W, rank, omap, keys_total, total, dev, stream, directory):
    """The owner `rank`'s received batches for every step, as (local ids, permits, ts)."""
    from distributedratelimiting.redis_amd import cluster
    n = args.batch
    dmap = torch.from_numpy(np.ascontiguousarray(omap, dtype=np.uint8)).to(dev)
    work = torch.empty(max(1, lib.tbe_route_workspace_bytes(n, W)), dtype=torch.uint8, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.zeros(W, dtype=torch.int64, device=dev)
    out = []
    for s_ in range(total):
        parts = []
        for src in range(W):
            k, p, t = _gen(lib, SEED_C, keys_total, s_, (s_ * W + src) * n, n, args.interval_us, args.zipf_s,
                           dev, stream)
            assert lib.tbe_route_plan_map_device(k.data_ptr(), n, W, dmap.data_ptr(), work.data_ptr(), pos.data_ptr(),
                                                 counts.data_ptr(), stream) == 0
            send = torch.empty((n, 3), dtype=torch.int64, device=dev)
            assert lib.tbe_route_pack_device(pos.data_ptr(), n, k.data_ptr(), p.data_ptr(), t.data_ptr(),
                                             send.data_ptr(), stream) == 0
            c = counts.cpu().tolist()
            off = sum(c[:rank])
            parts.append(send[off:off + c[rank]].clone())
            del k, p, t, send
        recv = torch.cat(parts)
        del parts
        ids = directory.assign(recv[:, 0].contiguous())
        out.append((ids, recv[:, 2].to(torch.int32), recv[:, 1].contiguous()))
        del recv
    directory.check()
    return out


def time_owner(args, keys_local, bufs, dev):
    """The driver's schedule on one owner's batches: warm-up, then the timed steps between
    synchronisations; the engine as bench.py builds it (pipelined, hot runs).  The stage
    times are the pipelined engine's event intervals, so the two streams' stages overlap."""
    from distributedratelimiting.redis_amd import TokenBucketEngine
    m_max = max(b[0].numel() for b in bufs)
    eng = TokenBucketEngine(keys_local, args.token_limit, args.tokens_per_period, args.period_ticks,
                            device=dev.index, stage_timing=True, max_batch=m_max, fold_records=not args.unscatter_all,
                            digit_stream=not args.hist_records, rerank=args.rerank)
    g = torch.empty(m_max, dtype=torch.uint8, device=dev)
    r = torch.empty(m_max, dtype=torch.int32, device=dev)
    for s_ in range(args.warmup):
        m = bufs[s_][0].numel()
        eng.acquire_batch_device(*bufs[s_], g[:m], r[:m])
    eng.synchronize()
    torch.cuda.synchronize()
    eng.stage_times()
    t0 = time.perf_counter()
    for s_ in range(args.warmup, args.warmup + args.steps):
        m = bufs[s_][0].numel()
        eng.acquire_batch_device(*bufs[s_], g[:m], r[:m])
    eng.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = eng.stage_times()
    lay = eng.layout()
    eng.close()
    return elapsed / args.steps * 1e3, {k: round(v / args.steps, 4) for k, v in st.items()}, lay


def run(args, lib, dev):
    from distributedratelimiting.redis_amd import cluster
    W = args.emulate_world
    n = args.batch
    keys_total = (args.keys or 125_000_000) * W
    total = args.warmup + args.steps
    side = torch.cuda.Stream(dev)
    torch.cuda.set_stream(side)
    stream = side.cuda_stream
    # per-step virtual-node loads of the whole global stream
    t_start = time.perf_counter()
    vn = np.zeros((total, cluster.OWNER_MAP_SIZE), dtype=np.int64)
    for s_ in range(total):
        acc = torch.zeros(cluster.OWNER_MAP_SIZE, dtype=torch.int64, device=dev)
        for src in range(W):
            k = _gen(lib, SEED_C, keys_total, s_, (s_ * W + src) * n, n, args.interval_us, args.zipf_s, dev, stream,
                     keys_only=True)
            acc += cluster.vnode_loads(k)
        vn[s_] = acc.cpu().numpy()
    maps = {"hash": cluster.hash_owner_map(W), "balanced": cluster.balanced_owner_map(vn[0], W, n_keys=keys_total)}
    hot_vnode = int(np.argmax(vn[0]))
    res = {}
    for name, m in maps.items():
        loads = np.stack([np.bincount(m, weights=vn[s_], minlength=W) for s_ in range(total)]).astype(np.int64)
        timed = loads[args.warmup:]
        mean = timed.mean(axis=0)                       # per rank over the timed steps
        worst = int(np.argmax(mean))
        typical = int(np.argmin(np.abs(mean - mean.mean())))
        hot_owner = int(m[hot_vnode])
        pick = sorted({worst, typical, hot_owner})
        keys_local = cluster.keys_per_rank(keys_total, W, owner_map=m)
        ranks = {}
        for rk in pick:
            d = cluster.DeviceDirectory(keys_local, device=dev.index)
            bufs = owner_stream(lib, args, W, rk, m, keys_total, total, dev, stream, d)
            ms, st, lay = time_owner(args, keys_local, bufs, dev)
            ranks[str(rk)] = {"role": ",".join(x for x, y in (("max_load", worst), ("mean_load", typical),
                                                              ("hot_key_owner", hot_owner)) if y == rk),
                              "requests_per_step": round(float(mean[rk]), 1), "ms_per_step": round(ms, 4),
                              "stage_ms_per_step_overlapped": st, "directory_ids": d.size(),
                              "layout": lay}
            del bufs
            d.close()
            torch.cuda.empty_cache()
        slowest = max(ranks.values(), key=lambda x: x["ms_per_step"])
        res[name] = {"per_rank_requests_per_step": [round(float(x), 1) for x in mean],
                     "max_over_mean_load": round(float(mean.max() / mean.mean()), 4),
                     "keys_per_rank_capacity": keys_local,
                     "emulated_ranks": ranks,
                     "slowest_ms_per_step": slowest["ms_per_step"],
                     "slowest_over_mean_load_rank": round(slowest["ms_per_step"] / ranks[str(typical)]["ms_per_step"], 4),
                     "implied_node_decisions_per_s": round(W * n / (slowest["ms_per_step"] * 1e-3), 1)}
    return {
        "metric": "acquire decisions/sec (node) at 100M keys, 1/2/4/8 GPU; % HBM roofline",
        "value": res["balanced"]["implied_node_decisions_per_s"],
        "unit": "decisions/s",
        "n_gpus": W,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["balanced"]["slowest_ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Zipf(1.1) keys by rejection-inversion, splitmix64 counters, generated in HBM)",
        "emulation": (f"EMULATION on one GPU: config C's owners at {W} GPUs, one at a time -- each chosen owner's "
                      "received stream (every source rank's requests for it, in (source, arrival) order) through its "
                      "own directory and engine on the driver's schedule; value = W * 2^26 / the slowest emulated "
                      "owner's ms per step under the balanced owner map; no collective and no other rank on the chip"),
        "config": {"workload": f"TokenBucket Zipf({args.zipf_s}) over {keys_total} keys, {W} x 2^{n.bit_length() - 1} "
                               f"requests per step, owners emulated one at a time (config C)",
                   "keys_total": keys_total, "batch_per_gpu": n, "token_limit": args.token_limit,
                   "tokens_per_period": args.tokens_per_period, "period_ticks": args.period_ticks,
                   "interval_us": args.interval_us, "owner_maps": res,
                   "hot_vnode_share_step0": round(float(vn[0][hot_vnode] / vn[0].sum()), 4)},
        "wall_s": round(time.perf_counter() - t_start, 1),
    }
