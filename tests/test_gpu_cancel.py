"""GPU parity of queued-request cancellation (tbe_queue_cancel; CancelQueueState,
Q:480-506 / A:531-557) against the Python restatement's ``cancel`` (oracle/semantics.py):
waits fill the queues, a random subset of queued, already-finished and unknown request
ids is canceled (several per key, duplicates included), then the replenish tick drains
what is left.  The queue contents, qsum (seen through later admissions) and the drain log
must match exactly."""
import numpy as np
import pytest

from oracle.semantics import (NEWEST_FIRST, OLDEST_FIRST, ApproxClient, ApproxGlobalTable,
                              QueueingTokenBucketTable, TokenBucketConfig, approx_refresh_all)

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000


def pick_cancels(rng, keys, rid0, n, queued_by_key):
    """Mix of queued ids (on their key), ids on the wrong key, finished ids, duplicates."""
    ck, ci = [], []
    for k, ids in queued_by_key.items():
        for x in ids:
            if rng.random() < 0.4:
                ck.append(k)
                ci.append(x)
                if rng.random() < 0.1:          # second cancel of the same request
                    ck.append(k)
                    ci.append(x)
    for _ in range(n // 20):                    # any request of the batch, maybe not queued
        i = int(rng.integers(0, n))
        ck.append(int(keys[i]) if rng.random() < 0.7 else int(rng.integers(0, 1 + keys.max())))
        ci.append(rid0 + i)
    ck.append(int(keys[0]))
    ci.append(-5)                               # never a request id
    perm = rng.permutation(len(ck))
    return np.array(ck, dtype=np.uint64)[perm], np.array(ci, dtype=np.int64)[perm]


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
@pytest.mark.parametrize("n_keys,qlimit", [(25, 6), (3000, 16)])
def test_queue_cancel(engine_lib, gpu, order, n_keys, qlimit):
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine
    rng = np.random.default_rng(7 * n_keys + order + qlimit)
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0)
    ref = QueueingTokenBucketTable(TokenBucketConfig.from_options(4, 1, 10_000_000), qlimit, order)
    t, rid, total = S_US, 0, 0
    for step in range(6):
        n = 20 * n_keys
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        st, rem, _ = eng.wait_batch(keys, permits, ts, rid)
        exp = [ref.acquire(int(k), int(p), int(x), rid + i)
               for i, (k, p, x) in enumerate(zip(keys, permits, ts))]
        assert st.tolist() == [e[0] for e in exp]
        assert rem.tolist() == [e[1] for e in exp]
        queued = {k: [e.request_id for e in q] for k, q in ref.queues.items() if q}
        ck, ci = pick_cancels(rng, keys, rid, n, queued)
        got = eng.cancel(ck, ci)
        want = [ref.cancel(int(k), int(x)) for k, x in zip(ck, ci)]
        assert got.tolist() == [int(w) for w in want]
        total += int(got.sum())
        for k in range(0, n_keys, max(1, n_keys // 40)):
            assert eng.queue_of(k) == ref.queue_of(k)
        rid += n
        t += 700_000
        k1, i1, r1 = eng.refresh(t)
        assert list(zip(k1.tolist(), i1.tolist(), r1.tolist())) == ref.refresh(t)
        t += 1_000
    assert total > 0


def test_queue_cancel_errors(engine_lib, gpu):
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, TbeError, TokenBucketEngine
    eng = QueueingTokenBucketEngine(10, 4, 1, 10_000_000, 4, OLDEST_FIRST, device=0)
    assert eng.cancel(np.zeros(0, np.uint64), np.zeros(0, np.int64)).size == 0
    with pytest.raises(TbeError):
        eng.cancel(np.array([10], np.uint64), np.array([0], np.int64))
    tb = TokenBucketEngine(10, 4, 1, 10_000_000, device=0)
    with pytest.raises(TbeError):
        QueueingTokenBucketEngine.cancel(tb, np.array([0], np.uint64), np.array([0], np.int64))


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_approx_cancel(engine_lib, gpu, order):
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n, limit, tokens, ticks, qlimit = 200, 3000, 20, 10, 10_000_000, 8
    rng = np.random.default_rng(500 + order)
    eng = ApproximateEngine(n_keys, limit, tokens, ticks, qlimit, order, device=0)
    cli = ApproxClient(limit, tokens, ticks, qlimit, order)
    table = ApproxGlobalTable(cli.decay_rate)
    rid = 0
    for epoch in range(5):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 2, 3], n).astype(np.int32)
        st, av, _ = eng.acquire_batch(keys, permits, wait=True, id_base=rid)
        exp = [cli.wait(k, p, rid + i)[0] for i, (k, p) in enumerate(zip(keys.tolist(), permits.tolist()))]
        assert st.tolist() == exp
        queued = {k: [e.request_id for e in s.queue] for k, s in cli.keys.items() if s.queue}
        ck, ci = pick_cancels(rng, keys, rid, n, queued)
        got = eng.cancel(ck, ci)
        assert got.tolist() == [int(cli.cancel(int(k), int(x))) for k, x in zip(ck, ci)]
        rid += n
        ts = S_US + epoch * 1_000_000
        k1, i1, _ = eng.refresh(ts)
        exp_log = approx_refresh_all([cli], table, ts, 0, range(n_keys))[0]
        assert list(zip(k1.tolist(), i1.tolist())) == exp_log
        for key in range(0, n_keys, 9):
            lo, gl, est, a, q = eng.local_state(key)
            s = cli.st(key)
            assert (lo, gl, est, a, q) == (s.local, s.global_, s.est, cli.available(s), len(s.queue))
            assert [x for x, _ in eng.queue_of(key)] == [e.request_id for e in s.queue]


def test_queue_cancel_config_d_scale(engine_lib, gpu):
    """Config D's shape (QueueLimit 16, TokenLimit 4, 1M keys, 1M-request batch): cancel
    30% of the queued requests in one call (~1e5 key runs).  Size-independent checks:
    every one hits once, sampled queues lose exactly the canceled ids in order, a second
    cancel finds nothing, and the next tick never grants a canceled id."""
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine
    from oracle import trace
    n_keys, n = 1 << 20, 1 << 20
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 16, OLDEST_FIRST, device=0)
    for b in range(2):
        k, p, ts = trace.make_batch(0x5EED000D, n_keys, b, n, 1_000)
        st, _, _ = eng.wait_batch(k, p, ts, b * n)
    queued = np.flatnonzero(st == 2)
    assert queued.size > 1000
    rng = np.random.default_rng(9)
    pick = rng.choice(queued, queued.size * 3 // 10, replace=False)
    ck, ci = k[pick].astype(np.uint64), (n + pick).astype(np.int64)
    sample = np.unique(ck)[:: max(1, np.unique(ck).size // 200)]
    before = {int(x): eng.queue_of(int(x)) for x in sample}
    hit = eng.cancel(ck, ci)
    assert hit.all()
    gone = set(ci.tolist())
    for x, q in before.items():
        assert eng.queue_of(x) == [e for e in q if e[0] not in gone]
    assert not eng.cancel(ck, ci).any()
    _, ids, _ = eng.refresh(trace.T0_US + 3 * 1_000_000)
    assert ids.size > 0 and not gone & set(ids.tolist())


def test_approx_cancel_scale(engine_lib, gpu):
    """Approximate kind, 1M keys and 2M waits over 2 batches (caps exhausted, queues in
    use): cancel a third of the queued requests in one call; sampled queues lose exactly
    those ids, local state (qsum via `queued`) follows, and the next refresh never
    completes a canceled id."""
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n = 1 << 20, 1 << 20
    eng = ApproximateEngine(n_keys, 4, 4, 10_000_000, 8, OLDEST_FIRST, device=0)
    rng = np.random.default_rng(31)
    for b in range(2):
        k = rng.integers(0, n_keys, n).astype(np.uint64)
        p = rng.choice([1, 1, 2, 3], n).astype(np.int32)
        st, _, _ = eng.acquire_batch(k, p, wait=True, id_base=b * n)
    queued = np.flatnonzero(st == 2)
    assert queued.size > 1000
    pick = rng.choice(queued, queued.size // 3, replace=False)
    ck, ci = k[pick], (n + pick).astype(np.int64)
    uk = np.unique(ck)
    sample = uk[:: max(1, uk.size // 200)]
    before = {int(x): eng.queue_of(int(x)) for x in sample}
    assert eng.cancel(ck, ci).all()
    gone = set(ci.tolist())
    for x, q in before.items():
        left = [e for e in q if e[0] not in gone]
        assert eng.queue_of(x) == left
        assert eng.local_state(x)[4] == len(left)
    assert not eng.cancel(ck, ci).any()
    _, ids, _ = eng.refresh(S_US + 5_000_000)
    assert not gone & set(ids.tolist())
