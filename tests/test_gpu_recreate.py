"""Engines created after other engines were used and destroyed in the same process
(VERDICT r05 item 1).

Round 5 saw wrong replies from queue and approximate engines only when they were created
after another engine had been freed, and only while their rings were allocated physically
contiguous.  These tests pin the invariant that matters whatever the allocator does: a
fresh engine starts from its own initial state -- every bucket absent with TokenLimit
tokens, every queue empty, every local and global tier at its default -- and decides its
first batches exactly as a fresh C restatement does (Q:67-134, Q:237-271, A:84-214,
A:241-270).  The previous engines use the same sizes, seeds and inputs, so stale memory
of theirs would reproduce their own later state, which differs from the initial one."""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000
N_KEYS, N, NB = 200_000, 1 << 18, 4


def _dev(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _sorted_log(keyseq, ids, rem, count):
    m = int(count.item())
    ks = keyseq[:m].cpu().numpy().view(np.uint64)
    o = np.argsort(ks, kind="stable")
    return (ks[o] >> np.uint64(16)), ids[:m].cpu().numpy()[o], rem[:m].cpu().numpy()[o]


def _queue_engine(order, qlimit):
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine
    return QueueingTokenBucketEngine(N_KEYS, 4, 1, 10_000_000, qlimit, order, device=0)


def _queue_b2b(eng, gpu, order, qlimit, seed, check=True):
    """NB fused-tick batches back to back, no host synchronisation between them (as
    test_back_to_back_tick_batches); with check, every reply, drain log, the evictions,
    sampled queues and the table against a fresh C restatement."""
    import torch
    from distributedratelimiting.redis_amd import fill_rate
    rng = np.random.default_rng(seed)
    cap = N_KEYS * min(max(qlimit, 1), 4)
    t, host, ins, outs, logs = S_US, [], [], [], []
    for b in range(NB):
        keys = rng.integers(0, N_KEYS, N).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3], N).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, N))).astype(np.int64)
        t += 1_000 + (int(rng.integers(0, 3_000_000)) if b % 2 else 0)
        host.append((keys, permits, ts, t))
        ins.append((_dev(keys.view(np.int64), gpu), _dev(permits, gpu), _dev(ts, gpu)))
        outs.append((torch.full((N,), 255, dtype=torch.uint8, device=gpu),
                     torch.empty(N, dtype=torch.int32, device=gpu)))
        logs.append((torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
                     torch.empty(cap, dtype=torch.int32, device=gpu), torch.empty(1, dtype=torch.int32, device=gpu)))
    torch.cuda.synchronize()   # NULL stream: inputs complete at the call
    for b in range(NB):
        eng.wait_batch_tick_device(*ins[b], *outs[b], b * N, host[b][3], *logs[b])
    eng.synchronize()
    if not check:
        return
    ref = cref.CQueueingTokenBucket(N_KEYS, 4, fill_rate(1, 10_000_000), qlimit, order)
    cause, ids = eng.evicted()
    for b in range(NB):
        keys, permits, ts, tick = host[b]
        st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, b * N)
        st = outs[b][0].cpu().numpy()
        bad = np.flatnonzero((st != st2) | (outs[b][1].cpu().numpy() != rem2))
        assert bad.size == 0, f"batch {b}: {bad.size} replies differ, first at {bad[:6].tolist()}"
        k1, i1, r1 = _sorted_log(*logs[b])
        k2, i2, r2 = ref.refresh(tick)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2), f"batch {b} log"
    assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
    for k in range(0, N_KEYS, 997):
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


def _assert_queue_initial(eng):
    v, tt = eng.export_state()
    assert (tt == np.iinfo(np.int64).min).all(), f"{int((tt != np.iinfo(np.int64).min).sum())} rows present"
    assert (v == 4.0).all()
    for k in range(0, N_KEYS, 211):
        assert eng.queue_of(k) == []


def _approx_epochs(eng, ref, gpu, seed, epochs, n):
    """acquire (wait) -> collect -> one-client sync per epoch; with ref, every status,
    availability, eviction, drain log and the final tiers against the C restatement."""
    import torch
    rng = np.random.default_rng(seed)
    counts = torch.zeros(N_KEYS, dtype=torch.int32, device=gpu)
    d_st = torch.empty(n, dtype=torch.uint8, device=gpu)
    d_av = torch.empty(n, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()
    for e in range(epochs):
        keys = rng.integers(0, N_KEYS, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3], n).astype(np.int32)
        eng.acquire_batch_device(_dev(keys.view(np.int64), gpu), _dev(permits, gpu), d_st, d_av,
                                 wait=True, id_base=e * n)
        eng.synchronize()
        ts = S_US + (e + 1) * 100_000
        if ref is not None:
            s2, a2, _, _ = ref.acquire_batch(keys, permits, wait=True, id_base=e * n)
            st = d_st.cpu().numpy()
            bad = np.flatnonzero((st != s2) | (d_av.cpu().numpy() != a2))
            assert bad.size == 0, f"epoch {e}: {bad.size} replies differ, first at {bad[:6].tolist()}"
        eng.collect(counts)
        torch.cuda.synchronize()
        k1, i1, r1 = eng.sync(counts, 1, 0, ts, 0)
        if ref is not None:
            c2 = ref.collect()
            assert np.array_equal(counts.cpu().numpy(), c2), f"epoch {e} counts"
            for got, exp in zip((k1, i1, r1), ref.sync(c2, 1, 0, ts, 0)):   # key order, both
                assert np.array_equal(got, exp), f"epoch {e} drain log"
    if ref is not None:
        x = ref.export()
        v, p, t = eng.export_global()
        assert np.array_equal(t, x["t_us"])
        m = t != np.iinfo(np.int64).min
        assert np.array_equal(v[m].view(np.uint64), x["v"][m].view(np.uint64))
        assert np.array_equal(p[m].view(np.uint64), x["p"][m].view(np.uint64))
        for k in range(0, N_KEYS, 499):
            lo, gl, est, av, q = eng.local_state(k)
            assert (lo, gl, av, q) == (int(x["local"][k]), int(x["global"][k]), int(x["available"][k]),
                                       int(x["queued"][k]))
            assert est == x["est"][k]


@pytest.mark.parametrize("order,qlimit", [(0, 16), (1, 4)])
def test_queue_engine_after_destroyed_engines(engine_lib, gpu, order, qlimit):
    """Create, use and destroy a queue engine and an approximate engine of the same sizes,
    then create the queue engine again: its table and queues are the initial ones before
    its first batch, and the back-to-back fused-tick sequence decides exactly as a fresh
    restatement, twice over (a third engine after the second is destroyed)."""
    from distributedratelimiting.redis_amd import ApproximateEngine
    seed = 4242 + order * 10 + qlimit
    first = _queue_engine(order, qlimit)
    _queue_b2b(first, gpu, order, qlimit, seed, check=False)
    first.close()
    a = ApproximateEngine(N_KEYS, 20, 10, 10_000_000, 8, order, device=0)
    _approx_epochs(a, None, gpu, seed, 2, N)
    a.close()
    for _ in range(2):
        eng = _queue_engine(order, qlimit)
        _assert_queue_initial(eng)
        _queue_b2b(eng, gpu, order, qlimit, seed, check=True)
        eng.close()


def test_approx_engine_after_destroyed_engines(engine_lib, gpu):
    """The same for the approximate kind: after an approximate and a queue engine were used
    and destroyed, a new approximate engine's global replica is absent everywhere and its
    local tiers are the defaults before its first batch, and three epochs decide exactly as
    a fresh restatement."""
    from distributedratelimiting.redis_amd import ApproximateEngine
    seed = 777
    a = ApproximateEngine(N_KEYS, 20, 10, 10_000_000, 8, 0, device=0)
    _approx_epochs(a, None, gpu, seed, 2, N)
    a.close()
    q = _queue_engine(0, 16)
    _queue_b2b(q, gpu, 0, 16, seed, check=False)
    q.close()
    for _ in range(2):
        eng = ApproximateEngine(N_KEYS, 20, 10, 10_000_000, 8, 0, device=0)
        ref = cref.CApprox(N_KEYS, 20, 10, 10_000_000, 8, 0, 4)
        v, p, t = eng.export_global()
        assert (t == np.iinfo(np.int64).min).all()
        x = ref.export()
        for k in range(0, N_KEYS, 211):
            lo, gl, est, av, qn = eng.local_state(k)
            assert (lo, gl, av, qn) == (int(x["local"][k]), int(x["global"][k]), int(x["available"][k]), 0)
            assert est == x["est"][k]
        _approx_epochs(eng, ref, gpu, seed, 3, N)
        eng.close()
