"""TokenBucketWithQueue spec: Python and C restatements agree, plus hand-checked cases."""
import numpy as np
import pytest

from oracle import cref
from oracle.semantics import (NEWEST_FIRST, OLDEST_FIRST, ST_FAILED, ST_GRANTED, ST_QUEUED,
                              ST_REJECTED, QueueingTokenBucketTable, TokenBucketConfig)

S_US = 1_760_572_800 * 1_000_000


def test_oldest_first_hand_case():
    q = QueueingTokenBucketTable(TokenBucketConfig(4, 1.0), 3, OLDEST_FIRST)
    out = [q.acquire(1, p, S_US + i, i) for i, p in enumerate([2, 2, 1, 1, 1, 1, 5])]
    assert [o[0] for o in out] == [ST_GRANTED, ST_GRANTED, ST_QUEUED, ST_QUEUED, ST_QUEUED,
                                   ST_FAILED, ST_REJECTED]
    assert out[2][1] == 0 and out[3][1] == -1          # script ran / not called
    assert q.refresh(S_US + 2_000_000) == [(1, 2, 1), (1, 3, 0)]
    assert q.queue_of(1) == [(4, 1)]


def test_newest_first_evicts_oldest():
    q = QueueingTokenBucketTable(TokenBucketConfig(2, 1.0), 3, NEWEST_FIRST)
    out = [q.acquire(1, p, S_US, i) for i, p in enumerate([2, 1, 1, 1, 2])]
    assert [o[0] for o in out] == [ST_GRANTED, ST_QUEUED, ST_QUEUED, ST_QUEUED, ST_QUEUED]
    assert out[4][2] == [1, 2]                          # evicted ids, oldest first
    assert q.queue_of(1) == [(3, 1), (4, 2)]
    # NewestFirst drains from the tail (DQ PeekTail/DequeueTail)
    assert q.refresh(S_US + 2_000_000) == [(1, 4, 0)]
    assert q.queue_of(1) == [(3, 1)]


def random_ops(seed, n_keys, rounds, n):
    rng = np.random.default_rng(seed)
    t = S_US
    for r in range(rounds):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3, 9], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 300_000, n))).astype(np.int64)
        t += 300_000
        yield keys, permits, ts, t
        t += int(rng.integers(0, 400_000))


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
@pytest.mark.parametrize("qlimit", [0, 1, 4, 16])
def test_python_vs_c(oracle_lib, order, qlimit):
    n_keys = 50
    cfg = TokenBucketConfig.from_options(5, 2, 10_000_000)
    py = QueueingTokenBucketTable(cfg, qlimit, order)
    c = cref.CQueueingTokenBucket(n_keys, cfg.token_limit, cfg.fill_rate, qlimit, order)
    rid = 0
    for keys, permits, ts, t_refresh in random_ops(qlimit * 7 + order, n_keys, 6, 2000):
        exp = [py.acquire(int(k), int(p), int(s), rid + i) for i, (k, p, s) in enumerate(zip(keys, permits, ts))]
        st, rem, ev_cause, ev_id = c.acquire_batch(keys, permits, ts, rid)
        assert st.tolist() == [e[0] for e in exp]
        assert rem.tolist() == [e[1] for e in exp]
        exp_ev = [(i, x) for i, e in enumerate(exp) for x in e[2]]
        assert list(zip(ev_cause.tolist(), ev_id.tolist())) == exp_ev
        rid += len(keys)
        lk, lid, lrem = c.refresh(t_refresh)
        assert list(zip(lk.tolist(), lid.tolist(), lrem.tolist())) == py.refresh(t_refresh)
    for k in range(n_keys):
        assert c.queue_of(k) == py.queue_of(k)


def test_cancel_hand_case():
    """CancelQueueState.TrySetCanceled (Q:480-506): qsum drops at once, the entry leaves
    the queue, a second cancel or a cancel of a finished request fails."""
    q = QueueingTokenBucketTable(TokenBucketConfig(4, 1.0), 3, OLDEST_FIRST)
    out = [q.acquire(1, p, S_US, i) for i, p in enumerate([4, 1, 2, 1])]
    assert [o[0] for o in out] == [ST_GRANTED, ST_QUEUED, ST_QUEUED, ST_FAILED]
    assert q.cancel(1, 1) and not q.cancel(1, 1) and not q.cancel(1, 0) and not q.cancel(2, 2)
    assert q.queue_of(1) == [(2, 2)] and q.qsum[1] == 2
    assert q.acquire(1, 1, S_US, 4)[0] == ST_QUEUED      # room freed by the cancel
    # the canceled head neither consumes tokens nor blocks: 2 s refill 2 tokens -> id 2 first
    assert q.refresh(S_US + 2_000_000) == [(1, 2, 0)]
    assert q.queue_of(1) == [(4, 1)]


def test_approx_cancel_hand_case():
    from oracle.semantics import AP_GRANTED, AP_QUEUED, ApproxClient
    c = ApproxClient(4, 4, 10_000_000, 4, OLDEST_FIRST)
    assert [c.wait(7, p, i)[0] for i, p in enumerate([4, 2, 2])] == [AP_GRANTED, AP_QUEUED, AP_QUEUED]
    assert c.cancel(7, 1) and not c.cancel(7, 1) and not c.cancel(8, 2)
    s = c.st(7)
    assert s.qcount == 2 and [e.request_id for e in s.queue] == [2]
    # the count is not added back to the local score (the A:489 double count)
    assert s.local == 4


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_cancel_invariants(order):
    """Random waits, cancels and ticks: qsum always equals the queued permits and stays
    within QueueLimit, a cancel never touches the bucket, and a canceled id never drains."""
    rng = np.random.default_rng(4242 + order)
    q = QueueingTokenBucketTable(TokenBucketConfig.from_options(4, 1, 10_000_000), 5, order)
    t, rid, canceled = S_US, 0, set()
    for step in range(40):
        for _ in range(30):
            k = int(rng.integers(0, 6))
            q.acquire(k, int(rng.choice([0, 1, 1, 2, 3])), t, rid)
            rid += 1
            t += int(rng.integers(0, 20_000))
        for k in range(6):
            for e in list(q.queues.get(k, [])):
                if rng.random() < 0.3:
                    before = q.tb.query(k)
                    assert q.cancel(k, e.request_id)
                    assert q.tb.query(k) == before
                    canceled.add(e.request_id)
        for k, ents in q.queues.items():
            assert q.qsum.get(k, 0) == sum(e.permits for e in ents) <= 5
        t += int(rng.integers(0, 900_000))
        assert not canceled & {x for _, x, _ in q.refresh(t)}
    assert canceled


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_c_queue_multithreaded_matches_serial(oracle_lib, order):
    """tbrq_*_mt (key-sharded, used by the full-size GPU parity tests) == serial tbrq_*:
    statuses, remaining, eviction logs (sorted by cause, id), tick logs and final state."""
    from distributedratelimiting.redis_amd import fill_rate
    n_keys, n = 3000, 40_000
    rate = fill_rate(2, 10_000_000)
    a = cref.CQueueingTokenBucket(n_keys, 4, rate, 6, order)
    b = cref.CQueueingTokenBucket(n_keys, 4, rate, 6, order)
    rng = np.random.default_rng(order + 5)
    t = S_US
    for r in range(4):
        k = rng.integers(0, n_keys, n).astype(np.uint64)
        p = rng.choice([0, 1, 1, 2, 3, 5], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 400_000, n))).astype(np.int64)
        t += 400_000
        sa, ra, ca, ia = a.acquire_batch(k, p, ts, r * n)
        sb, rb, cb, ib = b.acquire_batch(k, p, ts, r * n, threads=5)
        o = np.lexsort((ia, ca))
        assert np.array_equal(sa, sb) and np.array_equal(ra, rb)
        assert np.array_equal(ca[o], cb) and np.array_equal(ia[o], ib)
        la = a.refresh(t)
        lb = b.refresh(t, threads=7)
        for x, y in zip(la, lb):
            assert np.array_equal(x, y)
    for x, y in zip(a.bucket_state(), b.bucket_state()):
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64))
    for key in range(0, n_keys, 97):
        assert a.queue_of(key) == b.queue_of(key)


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_c_cancel_matches_python(oracle_lib, order):
    """tbrq_cancel (the C restatement the large sharded GPU tests use as their reference)
    against QueueingTokenBucketTable.cancel: queued, finished, unknown and repeated ids,
    between wait batches and ticks; queues and drain logs stay identical."""
    n_keys, qlimit = 40, 6
    cfg = TokenBucketConfig.from_options(5, 2, 10_000_000)
    py = QueueingTokenBucketTable(cfg, qlimit, order)
    c = cref.CQueueingTokenBucket(n_keys, cfg.token_limit, cfg.fill_rate, qlimit, order)
    rng = np.random.default_rng(5 + order)
    rid = 0
    for keys, permits, ts, t_refresh in random_ops(11 + order, n_keys, 6, 1500):
        for i, (k, p, s) in enumerate(zip(keys, permits, ts)):
            py.acquire(int(k), int(p), int(s), rid + i)
        c.acquire_batch(keys, permits, ts, rid)
        pick = rng.integers(0, len(keys), 300)
        ck, cid = keys[pick], rid + pick.astype(np.int64)
        cid[::7] = -5                                       # unknown ids
        want = [int(py.cancel(int(k), int(i))) for k, i in zip(ck, cid)]
        assert c.cancel(ck, cid).tolist() == want
        assert sum(want) > 0
        rid += len(keys)
        lk, lid, lrem = c.refresh(t_refresh)
        assert list(zip(lk.tolist(), lid.tolist(), lrem.tolist())) == py.refresh(t_refresh)
    for k in range(n_keys):
        assert c.queue_of(k) == py.queue_of(k)


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_c_approx_cancel_matches_python(oracle_lib, order):
    """tba_cancel against ApproxClient.cancel, zero-permit entries included."""
    from oracle.semantics import ApproxClient
    n_keys, qlimit = 30, 5
    py = ApproxClient(6, 3, 10_000_000, qlimit, order, zero_slots=2)
    c = cref.CApprox(n_keys, 6, 3, 10_000_000, qlimit, order, zero_slots=2)
    rng = np.random.default_rng(17 + order)
    rid = 0
    for _ in range(4):
        keys = rng.integers(0, n_keys, 800).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3], 800).astype(np.int32)
        for i, (k, p) in enumerate(zip(keys.tolist(), permits.tolist())):
            py.wait(k, p, rid + i)
        c.acquire_batch(keys, permits, wait=True, id_base=rid)
        pick = rng.integers(0, 800, 200)
        want = [int(py.cancel(int(keys[j]), rid + int(j))) for j in pick]
        assert c.cancel(keys[pick], rid + pick.astype(np.int64)).tolist() == want
        assert sum(want) > 0
        rid += 800
        for k in range(n_keys):
            s = py.st(k)
            assert c.queue_of(k) == [(e.request_id, e.permits) for e in s.queue]
