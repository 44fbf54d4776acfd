"""Config C's owners at the batch size an 8-GPU node gives them.

Config C is one global Zipf(1.1) stream over 1e9 keys, 8 x 2^26 requests per step, sharded
to 8 owners.  The owner of the hottest key (10.7% of the stream) receives
~1.08e8 requests per step under the hash partition; under the capped balanced owner map
the busiest owner still receives ~7.2e7.  Both exceed 2^26, the largest batch the
full-shape tests ran, and a batch above 2^26 changes the fold-record bit budget: the
reply position takes ceil_log2(n) = 27 bits and leaves fewer time-offset bits
(csrc/tbe_engine.hip FoldFmt).

These tests generate that global stream on the device exactly as bench_emul.py does (the
generators and draw order of bench.py's ranks), take the busiest owner's received stream
-- every source rank's requests for it, in (source, arrival) order, what
cluster.route_requests delivers -- through that owner's key directory, and run 4 steps
through a TokenBucketEngine whose max_batch is that size (steps 0 and 1 are the
cold-start sampling batches).  Every reply and the owned table are compared with the C
restatement (oracle/tb_ref.c, key-sharded threads) on the directory's ids
(PTB:42, TB:202-238)."""
import os
import time
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))
W, N, STEPS = 8, 1 << 26, 4
KEYS_TOTAL = 125_000_000 * W
ABSENT = np.iinfo(np.int64).min


def log(msg):
    print(f"[emul-owner {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _assert_no_escape(ts, bits):
    """Every request's time offset fits `bits` around the batch's first timestamp (PackFmt /
    FoldFmt base = ts[0] - 2^(bits-1)): the records ran in their non-escaped form."""
    d = ts.astype(np.int64) - (int(ts[0]) - (1 << (bits - 1)))
    assert d.min() >= 0 and d.max() < (1 << bits), (bits, int(d.min()), int(d.max()))


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("map_kind", ["hash", "balanced"])
def test_config_c_busiest_owner_at_8_gpus(engine_lib, gpu, map_kind):
    import torch
    import bench_emul
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, cluster, fill_rate
    lib = _capi.load()
    args = SimpleNamespace(batch=N, interval_us=10_000, zipf_s=1.1)
    side = torch.cuda.Stream(gpu)
    torch.cuda.set_stream(side)
    stream = side.cuda_stream
    try:
        vn0 = torch.zeros(cluster.OWNER_MAP_SIZE, dtype=torch.int64, device=gpu)
        for src in range(W):   # step 0's virtual-node loads of the whole global stream
            k = bench_emul._gen(lib, bench_emul.SEED_C, KEYS_TOTAL, 0, src * N, N, args.interval_us, args.zipf_s,
                                gpu, stream, keys_only=True)
            vn0 += cluster.vnode_loads(k)
        vn0 = vn0.cpu().numpy()
        omap = cluster.hash_owner_map(W) if map_kind == "hash" else \
            cluster.balanced_owner_map(vn0, W, n_keys=KEYS_TOTAL)
        loads = np.bincount(omap, weights=vn0, minlength=W)
        rank = int(np.argmax(loads))
        keys_local = cluster.keys_per_rank(KEYS_TOTAL, W, owner_map=omap)
        log(f"{map_kind} map: owner {rank} receives {int(loads[rank])} requests in step 0 "
            f"(max/mean {loads.max() / loads.mean():.3f}); table {keys_local} keys")
        d = cluster.DeviceDirectory(keys_local, device=0)
        bufs = bench_emul.owner_stream(lib, args, W, rank, omap, KEYS_TOTAL, STEPS, gpu, stream, d)
        torch.cuda.synchronize()
        sizes = [b[0].numel() for b in bufs]
        assert min(sizes) > (1 << 26), sizes          # the shape no earlier test ran
        if map_kind == "hash":
            assert min(sizes) > 100_000_000, sizes
        eng = TokenBucketEngine(keys_local, 10, 1, 10_000_000, device=0, max_batch=max(sizes), stage_timing=True)
        lay = eng.layout()
        assert lay["packed"] and lay["hot"] and lay["fold_records"] and lay["passes"] == 2, lay
        ref = cref.CTokenBucket(keys_local, 10, fill_rate(1, 10_000_000))
        g = torch.empty(max(sizes), dtype=torch.uint8, device=gpu)
        r = torch.empty(max(sizes), dtype=torch.int32, device=gpu)
        hot_ms, fold_ms = [], []
        for s_, (ids, p, t) in enumerate(bufs):
            m = ids.numel()
            fmt = eng.batch_format(m)
            assert fmt["fold_records"] and fmt["position_bits"] == 27, fmt
            assert fmt["fold_time_bits"] == 64 - fmt["r_bits"] - fmt["permit_bits"] - 1 - 27 >= 8, fmt
            eng.acquire_batch_device(ids, p, t, g[:m], r[:m], stream=stream)
            side.synchronize()
            eng.synchronize()
            st = eng.stage_times()
            hot_ms.append(st.get("hot", 0.0))
            fold_ms.append(st.get("fold", 0.0))
            hk = ids.cpu().numpy().view(np.uint64)
            hp = p.cpu().numpy()
            ht = t.cpu().numpy()
            assert hk.max() < keys_local
            _assert_no_escape(ht, fmt["pass0_time_bits"])
            _assert_no_escape(ht, fmt["fold_time_bits"])
            g_ref, r_ref = ref.acquire_batch(hk, hp, ht, threads=THREADS)
            gg, rr = g[:m].cpu().numpy(), r[:m].cpu().numpy()
            bad = np.flatnonzero((gg != g_ref) | (rr != r_ref))
            assert bad.size == 0, (s_, bad.size, bad[:5], gg[bad[:5]], rr[bad[:5]], g_ref[bad[:5]], r_ref[bad[:5]])
            top = int(np.unique(hk[: 1 << 20], return_counts=True)[1].max()) * (m >> 20)
            log(f"{map_kind} step {s_}: {m} replies identical (grant rate {g_ref.mean():.4f}, hottest key "
                f"~{top} requests; fold {fold_ms[-1]:.2f} ms, hot runs {hot_ms[-1]:.2f} ms; "
                f"position bits {fmt['position_bits']}, time bits {fmt['fold_time_bits']})")
        assert min(hot_ms) > 0.05, hot_ms            # hot runs from the cold-start batches on
        v, t_us = eng.export_state()
        v_ref, t_ref = ref.export_state()
        assert np.array_equal(t_us, t_ref), np.flatnonzero(t_us != t_ref)[:10]
        touched = t_ref != ABSENT
        assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
        log(f"{map_kind}: owner table ({keys_local} rows, {int(touched.sum())} written) identical")
        eng.close()
        d.close()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(gpu))


@pytest.mark.timeout(600)
def test_batch_above_2p26_with_escapes(engine_lib, gpu):
    """A 1.1e8-request batch over 1.25e8 keys whose timestamps span two hours: past +-35
    minutes the pass-0 records escape to the caller's timestamps (by a 27-bit arrival
    index), and past the fold record's +-0.5 s nearly every fold record escapes to its
    pass-0 record (by a 27-bit position).  Replies and table against the C restatement."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, fill_rate
    lib = _capi.load()
    n_keys, n = 125_000_000, 110_000_000
    span = 2 * 3600 * 1_000_000
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n)
    fmt = eng.batch_format(n)
    assert fmt["position_bits"] == 27 and fmt["fold_records"], fmt
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    k = torch.empty(n, dtype=torch.int64, device=gpu)
    p = torch.empty(n, dtype=torch.int32, device=gpu)
    t = torch.empty(n, dtype=torch.int64, device=gpu)
    g = torch.empty(n, dtype=torch.uint8, device=gpu)
    r = torch.empty(n, dtype=torch.int32, device=gpu)
    for b in range(2):
        assert lib.tbe_gen_batch_device(0x5EED0E5C, n_keys, b * n, n, 0, 3, 1_760_000_000_000_000 + b * span, span,
                                        k.data_ptr(), p.data_ptr(), t.data_ptr(), None) == 0
        torch.cuda.synchronize()
        eng.acquire_batch_device(k, p, t, g, r)
        eng.synchronize()
        ht = t.cpu().numpy()
        esc0 = ht - (int(ht[0]) - (1 << (fmt["pass0_time_bits"] - 1))) >= (1 << fmt["pass0_time_bits"])
        esc1 = ht - (int(ht[0]) - (1 << (fmt["fold_time_bits"] - 1))) >= (1 << fmt["fold_time_bits"])
        assert esc0.mean() > 0.4 and esc1.mean() > 0.9, (esc0.mean(), esc1.mean())
        g_ref, r_ref = ref.acquire_batch(k.cpu().numpy().view(np.uint64), p.cpu().numpy(), ht, threads=THREADS)
        gg, rr = g.cpu().numpy(), r.cpu().numpy()
        bad = np.flatnonzero((gg != g_ref) | (rr != r_ref))
        assert bad.size == 0, (b, bad.size, bad[:5])
        log(f"escape batch {b}: {n} replies identical ({esc0.mean():.2f} pass-0 and {esc1.mean():.2f} fold "
            f"records escaped)")
    v, t_us = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(t_us, t_ref)
    touched = t_ref != ABSENT
    assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
