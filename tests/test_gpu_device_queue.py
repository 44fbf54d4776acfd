"""GPU parity of the device-pointer queue and approximate entry points
(tbe_wait_batch_device, tbe_refresh_device, tbe_approx_acquire_batch_device): the same
traces as tests/test_gpu_queue.py / test_gpu_approx.py, inputs and replies in HBM, checked
against the C restatement (oracle/tb_ref.c) and the Python restatement (oracle/semantics.py),
including host-buffer calls made after device calls (the engine recounts its queues)."""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000


def _dev(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _sorted_log(keyseq, ids, rem, count):
    """Device drain log -> the host call's (key, drain order) listing."""
    m = int(count.item())
    ks = keyseq[:m].cpu().numpy().view(np.uint64)
    o = np.argsort(ks, kind="stable")
    return (ks[o] >> np.uint64(16)), ids[:m].cpu().numpy()[o], rem[:m].cpu().numpy()[o]


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("n_keys,qlimit,n,rounds", [(40, 4, 3000, 5), (5000, 16, 60000, 4), (7, 0, 2000, 3)])
def test_wait_and_refresh_device(engine_lib, gpu, order, n_keys, qlimit, n, rounds):
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    rng = np.random.default_rng(n_keys + 31 * qlimit + order + 7)
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0)
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), qlimit, order)
    t, rid = S_US, 0
    for rnd in range(rounds):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3, 5], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, rid)
        d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
        d_rem = torch.empty(n, dtype=torch.int32, device=gpu)
        eng.wait_batch_device(_dev(keys.view(np.int64), gpu), _dev(permits, gpu), _dev(ts, gpu),
                              d_st, d_rem, rid)
        eng.synchronize()
        assert np.array_equal(d_st.cpu().numpy(), st2)
        assert np.array_equal(d_rem.cpu().numpy(), rem2)
        cause, ids = eng.evicted()
        assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
        rid += n
        t += 1_000 + int(rng.integers(0, 3_000_000))
        k2, i2, r2 = ref.refresh(t)
        if rnd % 2 == 0:   # device drain
            cap = max(eng.refresh_bound(), 1)
            lk = torch.empty(cap, dtype=torch.int64, device=gpu)
            li = torch.empty(cap, dtype=torch.int64, device=gpu)
            lr = torch.empty(cap, dtype=torch.int32, device=gpu)
            cnt = torch.empty(1, dtype=torch.int32, device=gpu)   # the tick zeroes it on its stream
            eng.refresh_device(t, lk, li, lr, cnt)
            eng.synchronize()
            k1, i1, r1 = _sorted_log(lk, li, lr, cnt)
        else:              # host drain after device batches: the engine recounts its queues
            k1, i1, r1 = eng.refresh(t)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    for k in range(min(n_keys, 50)):
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


def test_refresh_device_capacity_checked(engine_lib, gpu):
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, TbeError
    eng = QueueingTokenBucketEngine(100, 2, 1, 10_000_000, 8, 0, device=0)
    n = 5000
    keys = np.arange(n, dtype=np.int64) % 100
    d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
    d_rem = torch.empty(n, dtype=torch.int32, device=gpu)
    ones, full = torch.ones(n, dtype=torch.int32, device=gpu), torch.full((n,), S_US, dtype=torch.int64, device=gpu)
    torch.cuda.synchronize()   # NULL stream: inputs must be complete at the call (include/tbe.h)
    eng.wait_batch_device(_dev(keys, gpu), ones, full, d_st, d_rem, 0)
    eng.synchronize()
    assert eng.refresh_bound() == 100 * 2   # n_keys * min(QueueLimit, TokenLimit)
    small = torch.empty(10, dtype=torch.int64, device=gpu)
    with pytest.raises(TbeError):
        eng.refresh_device(S_US + 1, small, small, small.view(torch.int32)[:10],
                           torch.empty(1, dtype=torch.int32, device=gpu))


def test_config_d_shape_device(engine_lib, gpu):
    """Config D shape (QueueLimit 16, OldestFirst, TokenLimit 4, 1 ms batches, refresh at
    each batch boundary) through the device entry points, as bench.py --workload queue."""
    import torch
    from oracle import trace
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    n_keys, n = 1_000_000, 1 << 20
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 16, 0, device=0)
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), 16, 0)
    cap = n_keys * 4
    lk = torch.empty(cap, dtype=torch.int64, device=gpu)
    li = torch.empty(cap, dtype=torch.int64, device=gpu)
    lr = torch.empty(cap, dtype=torch.int32, device=gpu)
    cnt = torch.empty(1, dtype=torch.int32, device=gpu)
    d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
    d_rem = torch.empty(n, dtype=torch.int32, device=gpu)
    for b in range(4):
        k, p, ts = trace.make_batch(0x5EED000D, n_keys, b, n, 1_000)
        st2, rem2, _, _ = ref.acquire_batch(k, p, ts, b * n)
        eng.wait_batch_device(_dev(k.view(np.int64), gpu), _dev(p, gpu), _dev(ts, gpu), d_st, d_rem, b * n)
        t_ref = trace.T0_US + (b + 1) * 1_000
        eng.refresh_device(t_ref, lk, li, lr, cnt)
        eng.synchronize()
        assert np.array_equal(d_st.cpu().numpy(), st2) and np.array_equal(d_rem.cpu().numpy(), rem2)
        k1, i1, r1 = _sorted_log(lk, li, lr, cnt)
        k2, i2, r2 = ref.refresh(t_ref)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    assert (st2 == 2).mean() > 0.05


@pytest.mark.parametrize("order,qlimit,wait", [(0, 8, True), (1, 4, True), (0, 0, False)])
def test_approx_acquire_device(engine_lib, gpu, order, qlimit, wait):
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    from oracle.semantics import ApproxClient, ApproxGlobalTable, approx_refresh_all
    n_keys, n, limit, tokens, ticks = 300, 4000, 20, 10, 10_000_000
    rng = np.random.default_rng(order * 10 + qlimit + 5)
    eng = ApproximateEngine(n_keys, limit, tokens, ticks, qlimit, order, device=0)
    client = ApproxClient(limit, tokens, ticks, qlimit, order)
    table = ApproxGlobalTable(client.decay_rate)
    counts = torch.zeros(n_keys, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()   # NULL stream: buffers complete at the call (include/tbe.h)
    d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
    d_av = torch.empty(n, dtype=torch.int32, device=gpu)
    rid = 0
    for epoch in range(5):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3, 25], n).astype(np.int32)
        eng.acquire_batch_device(_dev(keys.view(np.int64), gpu), _dev(permits, gpu), d_st, d_av,
                                 wait=wait, id_base=rid)
        eng.synchronize()
        exp, exp_ev = [], []
        for i, (k, p) in enumerate(zip(keys.tolist(), permits.tolist())):
            if wait:
                status, ev = client.wait(k, p, rid + i)
            else:
                status, ev = client.acquire(k, p), []
            exp.append((status, -1 if status == 3 else client.available(client.st(k))))
            exp_ev += [(i, x) for x in ev]
        assert d_st.cpu().tolist() == [x[0] for x in exp]
        assert d_av.cpu().tolist() == [x[1] for x in exp]
        cause, ids = eng.evicted()
        assert list(zip(cause.tolist(), ids.tolist())) == exp_ev
        rid += n
        ts = S_US + epoch * 1_000_000
        eng.collect(counts)
        k, i, _ = eng.sync(counts, 1, 0, ts, 0)   # host sync after device batches: recount
        exp_log = approx_refresh_all([client], table, ts, 0, range(n_keys))[0]
        assert list(zip(k.tolist(), i.tolist())) == exp_log
        for key in range(0, n_keys, 11):
            lo, gl, est, av, q = eng.local_state(key)
            s = client.st(key)
            assert (lo, gl, est, av, q) == (s.local, s.global_, s.est, client.available(s), len(s.queue))


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("n_keys,qlimit,n,rounds,sparse", [
    (5000, 16, 60000, 4, False),       # dense buckets (every row in LDS)
    (3_000_000, 4, 20000, 4, True),    # sparse and empty buckets: the tick still drains them
    (40, 4, 3000, 5, False),
])
def test_wait_batch_tick_device(engine_lib, gpu, order, n_keys, qlimit, n, rounds, sparse):
    """tbe_wait_batch_tick_device == tbe_wait_batch_device + tbe_refresh_device: replies,
    evictions, drain logs, queues and the bucket table, against the C restatement.  In the
    sparse case the keys queued by earlier rounds are mostly absent from later batches, so
    the drain runs in buckets that hold few or no requests."""
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    rng = np.random.default_rng(n_keys + 7 * qlimit + order)
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0)
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), qlimit, order)
    t, rid = S_US, 0
    hot = rng.integers(0, n_keys, 64).astype(np.uint64)
    for rnd in range(rounds):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        if sparse and rnd == 0:
            keys[: n // 2] = hot[rng.integers(0, 64, n // 2)]   # queues on a few keys first
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, rid)
        t += 1_000 + int(rng.integers(0, 3_000_000))
        k2, i2, r2 = ref.refresh(t)
        cap = max(n_keys * min(max(qlimit, 1), 4), 1)
        lk = torch.empty(cap, dtype=torch.int64, device=gpu)
        li = torch.empty(cap, dtype=torch.int64, device=gpu)
        lr = torch.empty(cap, dtype=torch.int32, device=gpu)
        cnt = torch.empty(1, dtype=torch.int32, device=gpu)
        d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
        d_rem = torch.empty(n, dtype=torch.int32, device=gpu)
        dk, dp, dt = _dev(keys.view(np.int64), gpu), _dev(permits, gpu), _dev(ts, gpu)
        torch.cuda.synchronize()   # NULL stream: inputs complete at the call
        eng.wait_batch_tick_device(dk, dp, dt, d_st, d_rem, rid, t, lk, li, lr, cnt)
        eng.synchronize()
        assert np.array_equal(d_st.cpu().numpy(), st2)
        assert np.array_equal(d_rem.cpu().numpy(), rem2)
        cause, ids = eng.evicted()
        assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
        k1, i1, r1 = _sorted_log(lk, li, lr, cnt)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
        rid += n
    for k in list(range(min(n_keys, 40))) + [int(x) for x in hot[:20]]:
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


@pytest.mark.parametrize("order,qlimit", [(0, 16), (1, 4)])
def test_back_to_back_tick_batches(engine_lib, gpu, order, qlimit):
    """Fused-tick queue batches enqueued back to back with no host synchronisation (as
    bench.py --workload queue) at a two-pass shape whose low-digit regions are a quarter
    tile (200,000 keys, 2^18 requests).  Every batch's statuses, remaining counts and
    drain log, the last batch's evictions, the queues and the bucket table against the C
    restatement (Q:67-134, Q:237-271)."""
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    n_keys, n, nb = 200_000, 1 << 18, 6
    rng = np.random.default_rng(order * 100 + qlimit)
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0)
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), qlimit, order)
    cap = n_keys * min(max(qlimit, 1), 4)
    t, host, ins, outs, logs = S_US, [], [], [], []
    for b in range(nb):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        t += 1_000 + (int(rng.integers(0, 3_000_000)) if b % 2 else 0)
        host.append((keys, permits, ts, t))
        ins.append((_dev(keys.view(np.int64), gpu), _dev(permits, gpu), _dev(ts, gpu)))
        outs.append((torch.empty(n, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu)))
        logs.append((torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
                     torch.empty(cap, dtype=torch.int32, device=gpu), torch.empty(1, dtype=torch.int32, device=gpu)))
    torch.cuda.synchronize()   # NULL stream: inputs complete at the call
    for b in range(nb):
        eng.wait_batch_tick_device(*ins[b], *outs[b], b * n, host[b][3], *logs[b])
    eng.synchronize()
    cause, ids = eng.evicted()
    for b in range(nb):
        keys, permits, ts, tick = host[b]
        st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, b * n)
        assert np.array_equal(outs[b][0].cpu().numpy(), st2), f"batch {b} statuses"
        assert np.array_equal(outs[b][1].cpu().numpy(), rem2), f"batch {b} remaining"
        k1, i1, r1 = _sorted_log(*logs[b])
        k2, i2, r2 = ref.refresh(tick)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2), f"batch {b} log"
    assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
    assert (st2 == 2).mean() > 0.05 and sum(int(lg[3].item()) for lg in logs) > 0
    for k in range(0, n_keys, 997):
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


@pytest.mark.parametrize("order", [0, 1])
def test_queue_narrow_pass0_with_escapes(engine_lib, gpu, order):
    """Round 6: the queueing kind's pass 0 writes 4-byte records (row | permit code | escape
    | time offset) beside the arrival index.  1e6 keys (r_bits 10) at TokenLimit 62 leave a
    15-bit time window (+-16 ms): batches spread over 4 s mostly escape (their times go to
    the side array), tight ones fit; fused ticks between them.  Statuses, remaining counts,
    evictions, drain logs, queues and the table against the C restatement (Q:67-134,
    Q:237-271)."""
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    n_keys, n, tl, ql = 1_000_000, 1 << 20, 62, 16
    eng = QueueingTokenBucketEngine(n_keys, tl, 5, 10_000_000, ql, order, device=0)
    assert eng.layout()["narrow_pass0"]
    assert eng.batch_format(n)["pass0_time_bits"] == 15
    ref = cref.CQueueingTokenBucket(n_keys, tl, fill_rate(5, 10_000_000), ql, order)
    rng = np.random.default_rng(17 + order)
    cap = n_keys * min(ql, tl)
    t = S_US
    for b, spread in enumerate([4_000_000, 1_000, 4_000_000, 20_000, 1_000]):
        keys = rng.integers(0, n_keys // 8, n).astype(np.uint64)     # ~8 requests per key
        permits = rng.choice([0, 1, 2, 7, 20, 63], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, spread, n))).astype(np.int64)
        if b == 2:
            ts = ts[::-1].copy()                                    # out of order
        t += spread + 500_000
        d = [_dev(keys.view(np.int64), gpu), _dev(permits, gpu), _dev(ts, gpu)]
        st = torch.empty(n, dtype=torch.uint8, device=gpu)
        rem = torch.empty(n, dtype=torch.int32, device=gpu)
        lg = (torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
              torch.empty(cap, dtype=torch.int32, device=gpu), torch.empty(1, dtype=torch.int32, device=gpu))
        torch.cuda.synchronize()
        eng.wait_batch_tick_device(*d, st, rem, b * n, t, *lg)
        eng.synchronize()
        st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, b * n, threads=8)
        bad = np.flatnonzero((st.cpu().numpy() != st2) | (rem.cpu().numpy() != rem2))
        assert bad.size == 0, (b, bad.size, bad[:5])
        cause, ids = eng.evicted()
        assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
        k1, i1, r1 = _sorted_log(*lg)
        k2, i2, r2 = ref.refresh(t, threads=8)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2), b
    for k in range(0, n_keys // 8, 1231):
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


def test_approx_narrow_pass0_acquire_then_wait(engine_lib, gpu):
    """Round 6: the approximate kind's AcquireCore batches take 4-byte pass-0 records (row |
    permit code; nothing reads an arrival index), its WaitAsync batches the 8-byte ones that
    carry it.  Both alternate on one engine at 1e6 keys; statuses, availability, evictions
    and sampled local tiers against the C restatement (A:84-214)."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n, tl = 1_000_000, 1 << 20, 40
    eng = ApproximateEngine(n_keys, tl, 10, 10_000_000, 6, 1, device=0)
    assert eng.layout()["narrow_pass0"]
    ref = cref.CApprox(n_keys, tl, 10, 10_000_000, 6, 1, 4)
    rng = np.random.default_rng(5)
    counts = torch.zeros(n_keys, dtype=torch.int32, device=gpu)
    d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
    d_av = torch.empty(n, dtype=torch.int32, device=gpu)
    for e, wait in enumerate([False, True, False, True, False]):
        keys = rng.integers(0, n_keys // 16, n).astype(np.uint64)
        permits = rng.choice([0, 1, 2, 5, 41], n).astype(np.int32)
        torch.cuda.synchronize()
        eng.acquire_batch_device(_dev(keys.view(np.int64), gpu), _dev(permits, gpu), d_st, d_av,
                                 wait=wait, id_base=e * n)
        eng.synchronize()
        s2, a2, c2, i2 = ref.acquire_batch(keys, permits, wait=wait, id_base=e * n, threads=8)
        bad = np.flatnonzero((d_st.cpu().numpy() != s2) | (d_av.cpu().numpy() != a2))
        assert bad.size == 0, (e, wait, bad.size, bad[:5])
        cause, ids = eng.evicted()
        assert np.array_equal(cause, c2) and np.array_equal(ids, i2)
        ts = S_US + (e + 1) * 1_000_000
        eng.collect(counts)
        torch.cuda.synchronize()
        got = eng.sync(counts, 1, 0, ts, 0)
        exp = ref.sync(ref.collect(), 1, 0, ts, 0, threads=8)
        for a, b in zip(got, exp):
            assert np.array_equal(a, b)
    x = ref.export()
    for k in range(0, n_keys // 16, 997):
        lo, gl, est, av, q = eng.local_state(k)
        assert (lo, gl, est, av, q) == (x["local"][k], x["global"][k], x["est"][k], x["available"][k],
                                        x["queued"][k])
