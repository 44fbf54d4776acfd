"""Full-shape GPU parity gate: every benchmarked configuration at the
size bench.py runs it, through the device entry points the bench uses (pipelined for the
token bucket), against the multithreaded C restatement (oracle/tb_ref.c) -- every reply,
every drain-log entry and the full final table, bit for bit.

  B  TokenBucket, 1e8 keys uniform, 2^26-request batches: 1375 requests per 2048-row
     bucket on average, so every bucket goes through k_fold_wide (TB:202-238)
  C  one GPU's slice of config C: 1.25e8 keys, Zipf(1.1) 2^26-request batches; from the
     third batch on the busiest keys take hot-key runs
  D  TokenBucketWithQueue, 1e8 keys, QueueLimit 16, OldestFirst, 1 ms batches + a
     replenish tick after each (Q:67-165, Q:237-271)

Sizes are the bench's; the oracle is key-sharded over the box's CPU share (16 threads),
so one batch checks in seconds."""
import os
import time

import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

T0_US = 1_760_000_000_000_000
ABSENT = np.iinfo(np.int64).min
THREADS = max(1, min(16, os.cpu_count() or 1))


def log(msg):
    print(f"[fullshape {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def assert_same_table(v, t, v_ref, t_ref):
    assert np.array_equal(t, t_ref), f"t_us mismatch at {np.flatnonzero(t != t_ref)[:10]}"
    touched = t_ref != ABSENT
    bad = np.flatnonzero(v[touched].view(np.uint64) != v_ref[touched].view(np.uint64))
    assert bad.size == 0, f"v mismatch at {np.flatnonzero(touched)[bad[:10]]}"


def assert_replies(b, g, r, g_ref, r_ref):
    bad = np.flatnonzero((g != g_ref) | (r != r_ref))
    assert bad.size == 0, (f"batch {b}: {bad.size} mismatches, first at {bad[:5]}: gpu "
                           f"{g[bad[:5]]},{r[bad[:5]]} ref {g_ref[bad[:5]]},{r_ref[bad[:5]]}")


@pytest.mark.timeout(900)
def test_config_b_full_shape_pipelined(engine_lib, gpu):
    """20 batches, as many as the driver's bench run (5 warm-up + 20 timed is 25): the
    table ages from all-grant (fresh keys) into the denial-dominated steady state
    (~67 requests per key per second against 1 token per second), so both the write-back
    of modified lines and the deny path are exercised at full size.  Batch b+1 is
    enqueued before batch b is checked, so its partition overlaps b's fold."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, fill_rate
    lib = _capi.load()
    n_keys, n, batches = 100_000_000, 1 << 26, 20
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n)
    lay = eng.layout()
    assert (lay["passes"], lay["r_bits"], lay["packed"], lay["pipeline"], lay["narrow"]) == (2, 11, True, True, True)
    nb = -(-n_keys // 2048)
    assert n // nb >= 1024, "uniform buckets must be full (k_fold_wide)"
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    sets = [tuple(torch.empty(n, dtype=dt, device=gpu) for dt in (torch.int64, torch.int32, torch.int64,
                                                                  torch.uint8, torch.int32)) for _ in range(2)]

    def enqueue(b):
        k, p, t, g, r = sets[b % 2]
        assert lib.tbe_gen_batch_device(0x5EED000B, n_keys, b * n, n, 1, 1, T0_US + b * 10_000, 10_000,
                                        k.data_ptr(), p.data_ptr(), t.data_ptr(), None) == 0
        torch.cuda.synchronize()
        eng.acquire_batch_device(k, p, t, g, r)

    def check(b):
        k, _, _, g, r = sets[b % 2]
        hk, hp, ht = cref.gen_batch(0x5EED000B, n_keys, b, n, 10_000)
        if b < 2:
            assert np.array_equal(k.cpu().numpy().view(np.uint64), hk)
        g_ref, r_ref = ref.acquire_batch(hk, hp, ht, threads=THREADS)
        assert_replies(b, g.cpu().numpy(), r.cpu().numpy(), g_ref, r_ref)
        if b % 4 == 0 or b == batches - 1:
            log(f"config B batch {b}: {n} replies identical (grant rate {g_ref.mean():.4f})")

    enqueue(0)
    for b in range(1, batches):
        enqueue(b)          # batch b's partition overlaps batch b-1's fold on the device
        eng.synchronize()
        check(b - 1)
    eng.synchronize()
    check(batches - 1)
    assert_same_table(*eng.export_state(), *ref.export_state())
    log("config B: 1e8-row table identical after 20 batches")


@pytest.mark.timeout(900)
def test_config_c_slice_full_shape(engine_lib, gpu):
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, fill_rate, workloads
    lib = _capi.load()
    n_keys, n, batches = 125_000_000, 1 << 26, 4
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n, stage_timing=True)
    assert eng.layout()["hot"]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    k = torch.empty(n, dtype=torch.int64, device=gpu)
    p = torch.ones(n, dtype=torch.int32, device=gpu)
    t = torch.empty(n, dtype=torch.int64, device=gpu)
    g = torch.empty(n, dtype=torch.uint8, device=gpu)
    r = torch.empty(n, dtype=torch.int32, device=gpu)
    hot_ms, fold_ms = [], []
    for b in range(batches):
        assert lib.tbe_gen_zipf_keys_device(0x5EED000C, n_keys, 1.1, b * n, n, k.data_ptr(), None) == 0
        ts = workloads.batch_timestamps(b, n, 10_000, T0_US)
        t.copy_(torch.from_numpy(ts))
        torch.cuda.synchronize()
        eng.acquire_batch_device(k, p, t, g, r)
        eng.synchronize()
        st = eng.stage_times()
        hot_ms.append(st.get("hot", 0.0))
        fold_ms.append(st.get("fold", 0.0))
        hk = k.cpu().numpy().view(np.uint64)
        g_ref, r_ref = ref.acquire_batch(hk, np.ones(n, np.int32), ts, threads=THREADS)
        assert_replies(b, g.cpu().numpy(), r.cpu().numpy(), g_ref, r_ref)
        top = int(np.unique(hk[: 1 << 20], return_counts=True)[1].max()) * 64
        log(f"config C batch {b}: {n} replies identical (grant rate {g_ref.mean():.4f}, "
            f"hottest key ~{top} requests, hot-run time {hot_ms[-1]:.3f} ms)")
    # hot runs exist from the first batch on: a key nominated by batch b's fold runs in b+2,
    # and the first two batches nominate their own dominant keys by sampling (cold start);
    # without that, their folds walked the hottest key's ~7.4M requests in one workgroup
    # (~27 ms each)
    assert min(hot_ms) > 0.05, hot_ms
    assert max(fold_ms) < 5.0, fold_ms
    assert_same_table(*eng.export_state(), *ref.export_state())
    log("config C slice: 1.25e8-row table identical")


def check_drain_log(b, m, lk, li, lr, ref_log):
    """A device drain log (key << 16 | drain position, request id, remaining; grouped
    arbitrarily across keys) against the C restatement's (key, drain) order."""
    ks = lk[:m].cpu().numpy().view(np.uint64)
    o = np.argsort(ks, kind="stable")
    lk_ref, li_ref, lr_ref = ref_log
    assert m == lk_ref.size, (b, m, lk_ref.size)
    assert np.array_equal(ks[o] >> np.uint64(16), lk_ref)
    assert np.array_equal(li[:m].cpu().numpy()[o], li_ref)
    assert np.array_equal(lr[:m].cpu().numpy()[o], lr_ref)


@pytest.mark.timeout(900)
def test_config_d_full_shape(engine_lib, gpu):
    """Config D as bench.py runs it: five 1 ms batches, each with its replenish tick
    fused into the fold (tbe_wait_batch_tick_device) -- at 1 token/s those ticks find no
    token for a saturated key -- then ticks that grant: standalone ticks
    (tbe_refresh_device) one second apart, each of which completes the head entry of
    every queue (Q:237-271), and a sixth batch whose fused tick also drains.  Statuses,
    remaining, every drain-log entry, the table and sampled queues against the C
    restatement (wait + refresh, tbrq_*)."""
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, _capi, fill_rate
    lib = _capi.load()
    n_keys, n, batches, tl, ql, interval = 100_000_000, 1 << 26, 5, 4, 16, 1_000
    eng = QueueingTokenBucketEngine(n_keys, tl, 1, 10_000_000, ql, 0, device=0, max_batch=n)
    ref = cref.CQueueingTokenBucket(n_keys, tl, fill_rate(1, 10_000_000), ql, 0)
    k = torch.empty(n, dtype=torch.int64, device=gpu)
    p = torch.empty(n, dtype=torch.int32, device=gpu)
    t = torch.empty(n, dtype=torch.int64, device=gpu)
    st = torch.empty(n, dtype=torch.uint8, device=gpu)
    rem = torch.empty(n, dtype=torch.int32, device=gpu)
    stream = torch.cuda.Stream(gpu)
    sh = stream.cuda_stream
    cap = n_keys * min(ql, tl)            # tbe_refresh_bound's ceiling: every key, min(QL, TL) grants
    lk = torch.empty(cap, dtype=torch.int64, device=gpu)
    li = torch.empty(cap, dtype=torch.int64, device=gpu)
    lr = torch.empty(cap, dtype=torch.int32, device=gpu)
    cnt = torch.empty(1, dtype=torch.int32, device=gpu)   # zeroed by the tick on its stream
    total_queued = 0
    drained = []

    def batch(b, ts0, tick):
        assert lib.tbe_gen_batch_device(0x5EED000D, n_keys, b * n, n, 1, 1, ts0, interval,
                                        k.data_ptr(), p.data_ptr(), t.data_ptr(), None) == 0
        torch.cuda.synchronize()
        eng.wait_batch_tick_device(k, p, t, st, rem, b * n, tick, lk, li, lr, cnt, stream=sh)
        stream.synchronize()
        hk, hp, ht = cref.gen_batch(0x5EED000D, n_keys, b, n, interval)
        ht = ht - (T0_US + b * interval) + ts0
        s_ref, r_ref, ev_c, _ = ref.acquire_batch(hk, hp, ht, b * n, threads=THREADS)
        assert ev_c.size == 0                                    # OldestFirst never evicts
        assert_replies(b, st.cpu().numpy(), rem.cpu().numpy(), s_ref, r_ref)
        m = int(cnt.item())
        check_drain_log(b, m, lk, li, lr, ref.refresh(tick, threads=THREADS))
        drained.append(m)
        log(f"config D batch {b}: {n} statuses identical ({int((s_ref == 1).sum())} granted, "
            f"{int((s_ref == 2).sum())} queued, {int((s_ref == 0).sum())} failed); fused tick drained {m}")
        return int((s_ref == 2).sum())

    for b in range(batches):
        total_queued += batch(b, T0_US + b * interval, T0_US + (b + 1) * interval)
    assert total_queued > 0
    # ticks that grant: a saturated key gains one token per second at 1 token/s
    for j in range(1, 4):
        tick = T0_US + j * 1_000_000
        eng.refresh_device(tick, lk, li, lr, cnt, stream=sh)
        stream.synchronize()
        m = int(cnt.item())
        check_drain_log(f"tick {j}", m, lk, li, lr, ref.refresh(tick, threads=THREADS))
        drained.append(m)
        log(f"config D standalone tick at T+{j} s: {m} queued entries completed, log identical")
    total_queued += batch(batches, T0_US + 4_000_000, T0_US + 5_000_000)
    # the granting ticks drain millions (at T+1 s only keys whose last grant is a full
    # second old have a token; from T+2 s on every queue's head)
    assert sum(drained[batches:]) > 10_000_000 and min(drained[batches + 1:]) > 1_000_000, drained
    v, t_us = eng.export_state()
    assert_same_table(v, t_us, *ref.bucket_state())
    rng = np.random.default_rng(4)
    for key in rng.integers(0, n_keys, 3000).tolist():
        assert eng.queue_of(key) == ref.queue_of(key)
    log(f"config D: {sum(drained)} drained entries, bucket table and 3000 sampled queues identical")


@pytest.mark.timeout(900)
def test_config_e_full_shape_two_clients(engine_lib, gpu):
    """Config E's shape: 1e7 shared keys, 2^26 AcquireCore requests per client per batch,
    then one refresh epoch (collect -> all-gather -> client-ordered sync replay with
    staggered timestamps, A:412-508) -- two client engines on one GPU, their counts
    concatenated exactly as RCCL's all-gather lays them out -- against two C
    restatements of the client (oracle/tb_ref.c tba_*): every status and AvailableTokens,
    the replica of the global tier and sampled local tiers, bit for bit."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine, _capi
    lib = _capi.load()
    kshared, n, tl, tpp, interval, clients, epochs = 10_000_000, 1 << 26, 100, 10, 10_000, 2, 3
    ticks = interval * 10
    engs = [ApproximateEngine(kshared, tl, tpp, ticks, 0, 0, device=0, max_batch=n) for _ in range(clients)]
    refs = [cref.CApprox(kshared, tl, tpp, ticks, 0, 0, 4) for _ in range(clients)]
    run_approx_epochs(gpu, engs, refs, kshared, n, interval, ticks, epochs, wait=False)


@pytest.mark.timeout(900)
def test_config_e_full_shape_queued_waits(engine_lib, gpu):
    """Config E's shape with QueueLimit 16 and WaitAsync (wait = 1): requests the local
    tier cannot lease queue (A:116-183), and every refresh epoch drains the queues in
    order while AvailableTokens covers the head (A:467-501) -- statuses, the drain logs,
    the global-tier replica and sampled local tiers against the C restatement."""
    from distributedratelimiting.redis_amd import ApproximateEngine
    kshared, n, tl, tpp, interval, clients, epochs, ql = 10_000_000, 1 << 26, 100, 10, 10_000, 2, 3, 16
    ticks = interval * 10
    engs = [ApproximateEngine(kshared, tl, tpp, ticks, ql, 0, device=0, max_batch=n) for _ in range(clients)]
    refs = [cref.CApprox(kshared, tl, tpp, ticks, ql, 0, 4) for _ in range(clients)]
    drained, queued = run_approx_epochs(gpu, engs, refs, kshared, n, interval, ticks, epochs, wait=True)
    assert queued > 1_000_000 and drained > 1_000_000, (queued, drained)


@pytest.mark.timeout(900)
def test_config_e_full_shape_eight_clients(engine_lib, gpu):
    """the refresh an 8-GPU node runs in config E -- 1e7 shared keys, 8
    clients, each client's counts all-gathered and every key's sync script replayed 8 times
    in client order with staggered timestamps (A:241-270, A:430-443) -- at full size: 8
    client engines (2^25 requests each per epoch), two epochs, every status, the whole
    global-tier replica and sampled local tiers against 8 C restatements (tba_*)."""
    from distributedratelimiting.redis_amd import ApproximateEngine
    kshared, n, tl, tpp, interval, clients, epochs = 10_000_000, 1 << 25, 100, 10, 10_000, 8, 2
    ticks = interval * 10
    engs = [ApproximateEngine(kshared, tl, tpp, ticks, 0, 0, device=0, max_batch=n) for _ in range(clients)]
    refs = [cref.CApprox(kshared, tl, tpp, ticks, 0, 0, 4) for _ in range(clients)]
    run_approx_epochs(gpu, engs, refs, kshared, n, interval, ticks, epochs, wait=False)


def run_approx_epochs(gpu, engs, refs, kshared, n, interval, ticks, epochs, wait):
    """Epochs of 2^26 requests per client, then collect -> the all-gather's layout ->
    client-ordered sync replay with staggered timestamps; returns (drained, queued)."""
    import torch
    from distributedratelimiting.redis_amd import _capi
    lib = _capi.load()
    clients = len(engs)
    k = torch.empty(n, dtype=torch.int64, device=gpu)
    p = torch.empty(n, dtype=torch.int32, device=gpu)
    t = torch.empty(n, dtype=torch.int64, device=gpu)
    st = torch.empty(n, dtype=torch.uint8, device=gpu)
    av = torch.empty(n, dtype=torch.int32, device=gpu)
    counts = [torch.empty(kshared, dtype=torch.int32, device=gpu) for _ in range(clients)]
    stagger = (ticks // 10) // clients
    drained = queued = 0
    for e in range(epochs):
        for r in range(clients):
            seed = 0x5EED000E + 7919 * r
            assert lib.tbe_gen_batch_device(seed, kshared, e * n, n, 1, 1, T0_US + e * interval, interval,
                                            k.data_ptr(), p.data_ptr(), t.data_ptr(), None) == 0
            torch.cuda.synchronize()
            engs[r].acquire_batch_device(k, p, st, av, wait=wait, id_base=e * n)
            engs[r].synchronize()
            hk = k.cpu().numpy().view(np.uint64)
            s_ref, a_ref, _, _ = refs[r].acquire_batch(hk, np.ones(n, np.int32), wait=wait, id_base=e * n,
                                                       threads=THREADS)
            assert_replies(e * clients + r, st.cpu().numpy(), av.cpu().numpy(), s_ref, a_ref)
            queued += int((s_ref == 2).sum())
            log(f"config E epoch {e} client {r}: {n} statuses identical (granted {(s_ref == 1).mean():.4f}, "
                f"queued {int((s_ref == 2).sum())})")
        for r in range(clients):
            engs[r].collect(counts[r])
        allc = torch.cat(counts)
        torch.cuda.synchronize()   # the engines' sync replay reads allc on their own streams
        allc_h = np.concatenate([ref.collect() for ref in refs])
        assert np.array_equal(allc.cpu().numpy(), allc_h)
        ts = T0_US + (e + 1) * interval
        for r in range(clients):
            got = engs[r].sync(allc, clients, r, ts, stagger)
            exp = refs[r].sync(allc_h, clients, r, ts, stagger, threads=THREADS)
            for a, b in zip(got, exp):                       # (key, request id, available) in key order
                assert np.array_equal(a, b)
            drained += got[0].size
            if not wait:
                assert got[0].size == 0                      # QueueLimit 0: nothing queued
        x = refs[0].export()
        v, pp, tt = engs[0].export_global()
        for a, b in ((v, x["v"]), (pp, x["p"]), (tt, x["t_us"])):
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
        for r in range(clients):
            x = refs[r].export()
            for key in np.random.default_rng(e * 10 + r).integers(0, kshared, 300).tolist():
                lo, gl, est, a, q = engs[r].local_state(key)
                assert (lo, gl, est, a, q) == (x["local"][key], x["global"][key], x["est"][key],
                                               x["available"][key], x["queued"][key])
                if wait and key % 10 == 0:
                    assert engs[r].queue_of(key) == refs[r].queue_of(key)
        log(f"config E epoch {e}: global tier replica (1e7 keys) and sampled local tiers identical "
            f"({drained} queued requests drained so far)")
    return drained, queued


@pytest.mark.timeout(900)
def test_key_turns_hot_mid_run(engine_lib, gpu):
    """a key that turns hot in a running engine.  Uniform 2^26-request
    batches over 1.25e8 keys; from batch 5 on, 10% of every batch (6.7M requests) is one key
    that was cold before.  Every batch is sampled (k_hot_sample), so the key runs apart in
    the very batch it turns hot -- no fold walks its millions of requests in one workgroup
    (~27 ms before) -- and replies and table stay identical to the C restatement."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, fill_rate
    lib = _capi.load()
    n_keys, n, batches, turn, hot_key = 125_000_000, 1 << 26, 8, 5, 98_765_432
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n, stage_timing=True)
    assert eng.layout()["hot"]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    k = torch.empty(n, dtype=torch.int64, device=gpu)
    p = torch.empty(n, dtype=torch.int32, device=gpu)
    t = torch.empty(n, dtype=torch.int64, device=gpu)
    g = torch.empty(n, dtype=torch.uint8, device=gpu)
    r = torch.empty(n, dtype=torch.int32, device=gpu)
    sel = (torch.arange(n, device=gpu) % 10) == 3
    for b in range(batches):
        assert lib.tbe_gen_batch_device(0x5EED00F0, n_keys, b * n, n, 1, 1, T0_US + b * 10_000, 10_000,
                                        k.data_ptr(), p.data_ptr(), t.data_ptr(), None) == 0
        if b >= turn:
            k[sel] = hot_key
        torch.cuda.synchronize()
        eng.acquire_batch_device(k, p, t, g, r)
        eng.synchronize()
        st = eng.stage_times()
        hk = k.cpu().numpy().view(np.uint64)
        g_ref, r_ref = ref.acquire_batch(hk, p.cpu().numpy(), t.cpu().numpy(), threads=THREADS)
        assert_replies(b, g.cpu().numpy(), r.cpu().numpy(), g_ref, r_ref)
        log(f"mid-run hot key, batch {b}: replies identical; fold {st.get('fold', 0):.3f} ms, "
            f"hot runs {st.get('hot', 0):.3f} ms")
        if b >= turn:
            assert st.get("fold", 0.0) < 5.0, (b, st)
            assert st.get("hot", 0.0) > 0.05, (b, st)
    assert_same_table(*eng.export_state(), *ref.export_state())
