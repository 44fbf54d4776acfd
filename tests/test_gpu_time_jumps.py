"""Timestamps hours apart (round 6).  The decision of the reference script (TB:202-238)
depends on the stored grant time exactly (refill and passive expiry), so these traces move
time by hours -- forward, backward, out of order inside a batch, one batch spanning seven
hours -- under a 10-hour TTL (rows stay present across the jumps), through dense folds,
sparse folds, hot-key runs and export -> import (the escaped-record paths: times outside a
batch's record window are read from the caller's array).  Every reply and the whole table
against the C restatement.  (Written for the 12-byte-row table that round 6 measured and
dropped, CHANGELOG round 6; they hold for any table layout.)"""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

T0 = 1_760_572_800 * 1_000_000
H = 3_600_000_000                 # one hour in us
ABSENT = np.iinfo(np.int64).min
THREADS = 8


def _rate():
    from distributedratelimiting.redis_amd import fill_rate
    return fill_rate(1, 36_000_000_000)   # 1 token per hour: TTL ceil(10 / rate) = 10 h


def _engine(n_keys, max_batch, **kw):
    from distributedratelimiting.redis_amd import TokenBucketEngine
    return TokenBucketEngine(n_keys, 10, 1, 36_000_000_000, device=0, max_batch=max_batch, **kw)


def _check(eng, ref, keys, permits, ts, tag):
    g, r = eng.acquire_batch(keys, permits, ts)
    g2, r2 = ref.acquire_batch(keys, permits, ts, threads=THREADS)
    bad = np.flatnonzero((g != g2) | (r != r2))
    assert bad.size == 0, (tag, bad.size, bad[:5], keys[bad[:5]], ts[bad[:5]])


def _check_table(eng, ref):
    v, t = eng.export_state()
    v2, t2 = ref.export_state()
    assert np.array_equal(t, t2), np.flatnonzero(t != t2)[:10]
    m = t2 != ABSENT
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


# (offset from T0 in us, spread of the batch in us, batch size, out of order)
SCHEDULE = [
    (0, 1_000, 1 << 20, False),             # dense: every bucket's epoch set
    (10_000, 5_000, 1 << 12, False),        # sparse
    (3 * H, 1_000, 1 << 20, False),         # +3 h: epochs move, the rows of 0 go to the side array
    (3 * H + 50_000, 2_000, 1 << 12, False),
    (H, 10_000, 1 << 20, True),             # back to +1 h, out of order: writes below the epochs
    (5 * H, 7 * H, 1 << 20, False),         # one batch spanning 7 hours
    (5 * H + 1, 1_000, 1 << 14, False),     # sparse again
    (20 * H, 1_000, 1 << 20, False),        # +20 h: every row has lapsed (TTL 10 h)
]


def test_time_jumps_dense_and_sparse(engine_lib, gpu):
    n_keys = 1_000_000                         # r_bits 10: dense batches of 2^20, sparse below
    eng = _engine(n_keys, 1 << 20)
    ref = cref.CTokenBucket(n_keys, 10, _rate())
    rng = np.random.default_rng(606)
    assert eng.batch_format(1 << 12)["sparse"] and not eng.batch_format(1 << 20)["sparse"]
    for i, (off, spread, n, ooo) in enumerate(SCHEDULE):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.integers(0, 4, n).astype(np.int32)
        ts = (T0 + off + np.sort(rng.integers(0, spread, n))).astype(np.int64)
        if ooo:
            rng.shuffle(ts)
        _check(eng, ref, keys, permits, ts, i)
        _check_table(eng, ref)
    eng.close()


def test_hot_keys_across_jumps(engine_lib, gpu):
    """Zipf batches whose hot keys run apart (k_hot_chain reads and writes their rows
    through the bucket epochs), with time jumping hours between them."""
    n_keys, n = 4_000_000, 1 << 22
    eng = _engine(n_keys, n)
    assert eng.layout()["hot"]
    ref = cref.CTokenBucket(n_keys, 10, _rate())
    rng = np.random.default_rng(77)
    perm = rng.permutation(1 << 20).astype(np.uint64) * 3 + 1
    for i, off in enumerate([0, 2 * H, 2 * H + 1_000, -H, 4 * H, 4 * H + 10]):
        ranks = np.minimum(rng.zipf(1.1, n), 1 << 20) - 1
        keys = perm[ranks]
        permits = rng.integers(0, 3, n).astype(np.int32)
        ts = (T0 + 2 * H + off + np.sort(rng.integers(0, 20_000, n))).astype(np.int64)
        _check(eng, ref, keys, permits, ts, i)
    _check_table(eng, ref)
    eng.close()


def test_export_import_with_side_rows(engine_lib, gpu):
    """A table whose rows span hours (some in the side array) exported and imported into a
    fresh engine -- whose buckets have no epoch yet, so every imported time starts in the
    side array -- then both engines decide the same batches as the restatement."""
    n_keys = 300_000
    a = _engine(n_keys, 1 << 19)
    ref = cref.CTokenBucket(n_keys, 10, _rate())
    rng = np.random.default_rng(5)
    for off in (0, 4 * H, 2 * H):
        keys = rng.integers(0, n_keys, 1 << 19).astype(np.uint64)
        permits = rng.integers(0, 4, 1 << 19).astype(np.int32)
        ts = (T0 + off + np.sort(rng.integers(0, 1_000, 1 << 19))).astype(np.int64)
        _check(a, ref, keys, permits, ts, off)
    v, t = a.export_state()
    b = _engine(n_keys, 1 << 19)
    b.import_state(v[:100_000], t[:100_000])
    b.import_state(v[100_000:], t[100_000:], first=100_000)
    v2, t2 = b.export_state()
    assert np.array_equal(t, t2) and np.array_equal(v[t != ABSENT].view(np.uint64), v2[t != ABSENT].view(np.uint64))
    for off in (4 * H + 5_000, 6 * H, 6 * H + 10):
        keys = rng.integers(0, n_keys, 1 << 19).astype(np.uint64)
        permits = rng.integers(0, 4, 1 << 19).astype(np.int32)
        ts = (T0 + off + np.sort(rng.integers(0, 1_000, 1 << 19))).astype(np.int64)
        ga, ra = a.acquire_batch(keys, permits, ts)
        gb, rb = b.acquire_batch(keys, permits, ts)
        g2, r2 = ref.acquire_batch(keys, permits, ts, threads=THREADS)
        assert np.array_equal(gb, g2) and np.array_equal(rb, r2), off
        assert np.array_equal(ga, g2) and np.array_equal(ra, r2), off
    _check_table(b, ref)
    va, ta = a.export_state()
    vb, tb = b.export_state()
    assert np.array_equal(ta, tb) and np.array_equal(va[ta != ABSENT].view(np.uint64), vb[tb != ABSENT].view(np.uint64))
    a.close()
    b.close()


def test_queue_time_jumps_with_fused_ticks(engine_lib, gpu):
    """The queueing kind (Q:67-134) with a replenish tick fused into every batch (Q:237-271)
    while time jumps by hours.  The folds derive request and row times on a 32-bit path
    relative to a base 2^31 us below each batch's first time, and fall back to the 64-bit
    derivation outside it (rows granted hours before, a batch spanning seven hours):
    statuses, remaining counts, evictions, drain logs, queues and the table against the C
    restatement.  1e6 keys at TokenLimit 4 give 40-bit record times (no escapes), so every
    fallback here is the time derivation's own."""
    import torch
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)

    n_keys, n, tl, ql = 1_000_000, 1 << 18, 4, 16
    for order in (0, 1):
        eng = QueueingTokenBucketEngine(n_keys, tl, 1, 36_000_000_000, ql, order, device=0, max_batch=n)
        ref = cref.CQueueingTokenBucket(n_keys, tl, fill_rate(1, 36_000_000_000), ql, order)
        rng = np.random.default_rng(91 + order)
        cap = n_keys * min(ql, tl)
        lg = (torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
              torch.empty(cap, dtype=torch.int32, device=gpu), torch.empty(1, dtype=torch.int32, device=gpu))
        for b, (off, spread, n_b, ooo) in enumerate(SCHEDULE):
            n_b = min(n_b, n)
            keys = rng.integers(0, n_keys // 4, n_b).astype(np.uint64)
            permits = rng.choice([0, 1, 1, 2, 3, 5], n_b).astype(np.int32)
            ts = (T0 + off + np.sort(rng.integers(0, spread, n_b))).astype(np.int64)
            if ooo:
                rng.shuffle(ts)
            t_tick = int(ts.max()) + 500_000
            st = torch.empty(n_b, dtype=torch.uint8, device=gpu)
            rem = torch.empty(n_b, dtype=torch.int32, device=gpu)
            d = [dev(keys.view(np.int64)), dev(permits), dev(ts)]
            torch.cuda.synchronize()
            eng.wait_batch_tick_device(*d, st, rem, b * n, t_tick, *lg)
            eng.synchronize()
            st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, b * n, threads=THREADS)
            bad = np.flatnonzero((st.cpu().numpy() != st2) | (rem.cpu().numpy() != rem2))
            assert bad.size == 0, (order, b, bad.size, bad[:5])
            cause, ids = eng.evicted()
            assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2), (order, b)
            m = int(lg[3].item())
            ks = lg[0][:m].cpu().numpy().view(np.uint64)
            o = np.argsort(ks, kind="stable")
            k2, i2, r2 = ref.refresh(t_tick, threads=THREADS)
            assert np.array_equal(ks[o] >> np.uint64(16), k2), (order, b)
            assert np.array_equal(lg[1][:m].cpu().numpy()[o], i2) and np.array_equal(lg[2][:m].cpu().numpy()[o], r2)
        for k in range(0, n_keys // 4, 4099):
            assert eng.queue_of(k) == ref.queue_of(k)
        v, tt = eng.export_state()
        v2, tt2 = ref.bucket_state()
        assert np.array_equal(tt, tt2)
        m = tt2 != ABSENT
        assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))
        eng.close()
