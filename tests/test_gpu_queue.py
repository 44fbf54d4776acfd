"""GPU parity of the TokenBucketWithQueue path (tbe_wait_batch / tbe_refresh) against the
C restatement of the spec (oracle/tb_ref.c tbrq_*), which tests/test_queue_oracle.py ties
to the Python restatement."""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000


def pair(n_keys, token_limit, tokens, ticks, qlimit, order):
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    eng = QueueingTokenBucketEngine(n_keys, token_limit, tokens, ticks, qlimit, order, device=0)
    ref = cref.CQueueingTokenBucket(n_keys, token_limit, fill_rate(tokens, ticks), qlimit, order)
    return eng, ref


def check_round(eng, ref, keys, permits, ts, id_base):
    st, rem, (cause, ids) = eng.wait_batch(keys, permits, ts, id_base)
    st2, rem2, cause2, ids2 = ref.acquire_batch(keys, permits, ts, id_base)
    bad = np.flatnonzero((st != st2) | (rem != rem2))
    assert bad.size == 0, f"{bad.size} mismatches at {bad[:5]}: {st[bad[:5]]} {rem[bad[:5]]} vs {st2[bad[:5]]} {rem2[bad[:5]]}"
    assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2)
    return st


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("n_keys,qlimit,n,rounds", [(40, 4, 3000, 5), (5000, 16, 60000, 4),
                                                    (1 << 20, 16, 200_000, 3), (7, 0, 2000, 3)])
def test_wait_and_refresh(engine_lib, gpu, order, n_keys, qlimit, n, rounds):
    rng = np.random.default_rng(n_keys + 31 * qlimit + order)
    eng, ref = pair(n_keys, 4, 1, 10_000_000, qlimit, order)
    t, rid = S_US, 0
    for _ in range(rounds):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3, 5], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        check_round(eng, ref, keys, permits, ts, rid)
        rid += n
        t += 1_000 + int(rng.integers(0, 3_000_000))
        k1, i1, r1 = eng.refresh(t)
        k2, i2, r2 = ref.refresh(t)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    for k in list(range(min(n_keys, 50))):
        assert eng.queue_of(k) == ref.queue_of(k)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("hot_share", [0.0, 0.01, 0.08, 0.5])
def test_tail_paths(engine_lib, gpu, order, hot_share):
    # k_fold_q after the first owner round (DESIGN.md §5 "tail walk"): few pending requests
    # and short runs take the walk; one key with tens to hundreds of requests per chunk
    # takes the rounds from the compacted list; more pending requests than threads keep
    # the register rounds.  Uniform keys plus one hot key at the given share.
    rng = np.random.default_rng(int(hot_share * 1000) + 7 * order)
    n_keys, n = 6000, 40_000
    eng, ref = pair(n_keys, 4, 1, 10_000_000, 16, order)
    t, rid = S_US, 0
    for _ in range(3):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        keys[rng.random(n) < hot_share] = 1234
        permits = rng.choice([0, 1, 1, 2, 3, 5], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        check_round(eng, ref, keys, permits, ts, rid)
        rid += n
        t += 2_000_000
        k1, i1, r1 = eng.refresh(t)
        k2, i2, r2 = ref.refresh(t)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    for k in [1234] + list(range(40)):
        assert eng.queue_of(k) == ref.queue_of(k)


def test_config_d_shape_small(engine_lib, gpu):
    # Config D shape: QueueLimit 16, OldestFirst, permits 1, TokenLimit 4, 1 ms batches,
    # demand >> fill so queues saturate; refresh at every batch boundary.
    from oracle import trace
    n_keys, n = 1_000_000, 1 << 20
    eng, ref = pair(n_keys, 4, 1, 10_000_000, 16, 0)
    for b in range(4):
        k, p, ts = trace.make_batch(0x5EED000D, n_keys, b, n, 1_000)
        st = check_round(eng, ref, k, p, ts, b * n)
        t_ref = trace.T0_US + (b + 1) * 1_000
        k1, i1, r1 = eng.refresh(t_ref)
        k2, i2, r2 = ref.refresh(t_ref)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    assert (st == 2).mean() > 0.05  # queues in use


@pytest.mark.parametrize("order", [0, 1])
def test_attempt_mixed_with_wait(engine_lib, gpu, order):
    """AttemptAcquire batches (tbe_queue_attempt_batch) interleaved with WaitAsync batches
    and replenish ticks, against the Python restatement (QueueingTokenBucketTable.attempt)."""
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine
    from oracle.semantics import QueueingTokenBucketTable, TokenBucketConfig
    rng = np.random.default_rng(99 + order)
    n_keys, qlimit = 30, 5
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0)
    ref = QueueingTokenBucketTable(TokenBucketConfig.from_options(4, 1, 10_000_000), qlimit, order)
    t, rid = S_US, 0
    for step in range(12):
        n = 400
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3, 5], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        if step % 3 == 1:
            st, rem = eng.attempt_batch(keys, permits, ts)
            exp = [ref.attempt(int(k), int(p), int(x)) for k, p, x in zip(keys, permits, ts)]
            assert st.tolist() == [e[0] for e in exp]
            assert rem.tolist() == [e[1] for e in exp]
            assert not (st == 2).any()
        else:
            st, rem, (cause, ids) = eng.wait_batch(keys, permits, ts, rid)
            exp = [ref.acquire(int(k), int(p), int(x), rid + i)
                   for i, (k, p, x) in enumerate(zip(keys, permits, ts))]
            assert st.tolist() == [e[0] for e in exp]
            assert rem.tolist() == [e[1] for e in exp]
            assert sorted(ids.tolist()) == sorted(i for e in exp for i in e[2])
            rid += n
        t += 700_000
        keys_l, ids_l, rem_l = eng.refresh(t)
        log = ref.refresh(t)
        assert list(zip(keys_l.tolist(), ids_l.tolist(), rem_l.tolist())) == log
        t += 1_000


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("layout", ["wide", "packed_wide_reply", "token_limit_100", "escaped_ts",
                                    "token_limit_16382", "token_limit_16383"])
def test_queue_layouts(engine_lib, gpu, order, layout):
    """The queue path's record and reply layouts against the C restatement: wide pass
    records (TBE_FLAG_NO_PACK), packed records with 4-byte replies (TBE_FLAG_NO_NARROW),
    TokenLimit 100 (too large for one-byte wait replies: two-byte ones), packed records whose
    timestamps leave the 32-bit window (escape records: the fold reads ts by index), and
    the two-byte replies' boundary: TokenLimit 16382 is the largest whose
    remaining fits 14 bits beside the "no script call" code 16383; 16383 takes four bytes."""
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate
    tl = int(layout.rsplit("_", 1)[1]) if layout.startswith("token_limit") else 4
    kw = {"wide": dict(pack=False, narrow=False), "packed_wide_reply": dict(narrow=False)}.get(layout, {})
    n_keys, n = 5000, 60_000
    eng = QueueingTokenBucketEngine(n_keys, tl, 1, 10_000_000, 16, order, device=0, **kw)
    ref = cref.CQueueingTokenBucket(n_keys, tl, fill_rate(1, 10_000_000), 16, order)
    lay = eng.layout()
    assert lay["packed"] == (layout != "wide") and lay["narrow"] == (layout in ("escaped_ts",))
    assert lay["medium"] == (layout in ("token_limit_100", "token_limit_16382"))
    rng = np.random.default_rng(hash(layout) % 1000 + order)
    t, rid = S_US, 0
    for _ in range(4):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        big = [tl // 3, tl // 2, tl] if tl > 100 else []
        permits = rng.choice([0, 1, 1, 2, 3, 5, tl + 1] + big, n).astype(np.int32)
        span = 3 * 3_600_000_000 if layout == "escaped_ts" else 1_000
        ts = (t + np.sort(rng.integers(0, span, n))).astype(np.int64)
        check_round(eng, ref, keys, permits, ts, rid)
        rid += n
        t = int(ts[-1]) + 1_000 + int(rng.integers(0, 3_000_000))
        k1, i1, r1 = eng.refresh(t)
        k2, i2, r2 = ref.refresh(t)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
    v, tt = eng.export_state()
    v2, tt2 = ref.bucket_state()
    assert np.array_equal(tt, tt2)
    m = tt2 != np.iinfo(np.int64).min
    assert np.array_equal(v[m].view(np.uint64), v2[m].view(np.uint64))


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("qlimit", [1024, 1025, 3000])
def test_long_queues_and_header_width(engine_lib, gpu, order, qlimit):
    """Queue headers are stored 32 bits wide up to QueueLimit 1024 (head 10 bits, count and
    queued permits 11) and 64 bits above: queues filled to the limit on both sides of the
    boundary -- a few keys, thousands of waits each, every permit count up to TokenLimit --
    with evictions (NewestFirst), replenish ticks, cancels and queue listings against the C
    restatement (Q:67-134, Q:237-271, Q:480-506)."""
    n_keys, n = 6, 20_000
    eng, ref = pair(n_keys, 7, 3, 10_000_000, qlimit, order)
    assert eng.queue_limit == qlimit and eng.layout()["queue_header_32"] == (qlimit <= 1024)
    rng = np.random.default_rng(qlimit * 2 + order)
    t, rid = S_US, 0
    for b in range(4):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([1, 1, 2, 3, 7, 8], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        st = check_round(eng, ref, keys, permits, ts, rid)
        if b == 1:
            assert (st == 2).any()
        rid += n
        t += 2_000_000 if b % 2 else 20_000
        k1, i1, r1 = eng.refresh(t)
        k2, i2, r2 = ref.refresh(t)
        assert np.array_equal(k1, k2) and np.array_equal(i1, i2) and np.array_equal(r1, r2)
        qs = [eng.queue_of(k) for k in range(n_keys)]
        assert qs == [ref.queue_of(k) for k in range(n_keys)]
        # cancel every fifth queued request of key 0 (and one unknown id)
        ids = [e[0] for e in qs[0][::5]] + [-7]
        ck = np.zeros(len(ids), dtype=np.uint64)
        c1 = eng.cancel(ck, np.array(ids, dtype=np.int64))
        c2 = ref.cancel(ck, np.array(ids, dtype=np.int64))
        assert np.array_equal(np.asarray(c1), np.asarray(c2))
    assert max(sum(p for _, p in q) for q in qs) > min(qlimit, 1024) // 2   # queues ran long
