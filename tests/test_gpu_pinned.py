"""tbe_alloc_host / tbe_free_host: host-buffer decisions from page-locked arrays equal
the ones from pageable arrays and the C restatement (oracle/tb_ref.c)."""
import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu


def test_pinned_host_buffers(engine_lib, gpu):
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    from distributedratelimiting.redis_amd.engine import PinnedArray
    n_keys, n = 50_000, 200_000
    pinned = [TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0),
              TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0)]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    bk, bp, bt = PinnedArray(n, np.uint64), PinnedArray(n, np.int32), PinnedArray(n, np.int64)
    for b in range(3):
        k, p, t = cref.gen_batch(0x5EED000B, n_keys, b, n, 10_000)
        bk.array[:], bp.array[:], bt.array[:] = k, p, t
        g1, r1 = pinned[0].acquire_batch(bk.array, bp.array, bt.array)
        g2, r2 = pinned[1].acquire_batch(k, p, t)
        g3, r3 = ref.acquire_batch(k, p, t)
        assert np.array_equal(g1, g3) and np.array_equal(r1, r3)
        assert np.array_equal(g2, g3) and np.array_equal(r2, r3)
    for a in (bk, bp, bt):
        a.free()
        a.free()                      # idempotent
    empty = PinnedArray(0, np.int64)
    assert empty.array.size == 0
    ref.close()


def test_pinned_chunked_overlap(engine_lib, gpu):
    """Batches of >= 2 chunks (4M requests each) from page-locked buffers take the chunked
    path (copies overlapping the decisions): same replies and table as the C restatement,
    including a ragged last chunk; an invalid request in the LAST chunk still rejects the
    whole batch with nothing applied."""
    from distributedratelimiting.redis_amd import TbeError, TokenBucketEngine, fill_rate
    from distributedratelimiting.redis_amd.engine import PinnedArray
    n_keys, n = 3_000_000, (1 << 24) + 12_345
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0)
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    bufs = [PinnedArray(n, d) for d in (np.uint64, np.int32, np.int64, np.uint8, np.int32)]
    bk, bp, bt, bg, br = (b.array for b in bufs)
    for b in range(3):
        k, p, t = cref.gen_batch(0x5EED000B, n_keys, b, n, 10_000, 1, 3)
        bk[:], bp[:], bt[:] = k, p, t
        g, r = eng.acquire_batch(bk, bp, bt, bg, br)
        g3, r3 = ref.acquire_batch(k, p, t, threads=8)
        assert np.array_equal(g, g3) and np.array_equal(r, r3), b
    v, tt = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(tt, t_ref)
    touched = t_ref != np.iinfo(np.int64).min
    assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
    k, p, t = cref.gen_batch(0x5EED000B, n_keys, 3, n, 10_000, 1, 3)
    bk[:], bp[:], bt[:] = k, p, t
    bp[n - 5] = -1
    with pytest.raises(TbeError):
        eng.acquire_batch(bk, bp, bt, bg, br)
    v2, t2 = eng.export_state()
    assert np.array_equal(t2, tt) and np.array_equal(v2.view(np.uint64), v.view(np.uint64))
    for a in bufs:
        a.free()
    ref.close()


@pytest.mark.parametrize("order", [0, 1])
def test_pinned_chunked_queue_and_approx(engine_lib, gpu, order):
    """Queue waits and approximate waits from page-locked buffers of >= 2 chunks take the
    chunked path: statuses, remaining / available and the eviction list (causes are
    offsets in the whole batch) equal the C restatement; an invalid request in the last
    chunk rejects the whole batch with nothing applied."""
    from distributedratelimiting.redis_amd import (ApproximateEngine, QueueingTokenBucketEngine, TbeError,
                                                   fill_rate)
    from distributedratelimiting.redis_amd.engine import PinnedArray
    n_keys, n = 2_000_000, (1 << 23) + 4_321
    bufs = [PinnedArray(n, d) for d in (np.uint64, np.int32, np.int64, np.uint8, np.int32)]
    bk, bp, bt, bs, br = (b.array for b in bufs)
    q = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 4, order, device=0)
    qref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), 4, order)
    a = ApproximateEngine(n_keys, 6, 1, 10_000_000, 4, order, device=0)
    aref = cref.CApprox(n_keys, 6, 1, 10_000_000, 4, order)
    for b in range(3):
        k, p, t = cref.gen_batch(0x5EED000D, n_keys, b, n, 1_000, 1, 3)
        bk[:], bp[:], bt[:] = k, p, t
        st, rem, (cause, ids) = q.wait_batch(bk, bp, bt, b * n, bs, br)
        st2, rem2, cause2, ids2 = qref.acquire_batch(k, p, t, b * n, threads=8)
        assert np.array_equal(st, st2) and np.array_equal(rem, rem2), b
        assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2), b
        st, av, (cause, ids) = a.acquire_batch(bk, bp, wait=True, id_base=b * n, status=bs, available=br)
        st2, av2, cause2, ids2 = aref.acquire_batch(k, p, True, b * n, threads=8)
        assert np.array_equal(st, st2) and np.array_equal(av, av2), b
        assert np.array_equal(cause, cause2) and np.array_equal(ids, ids2), b
    v, tt = q.export_state()
    k, p, t = cref.gen_batch(0x5EED000D, n_keys, 3, n, 1_000, 1, 3)
    bk[:], bp[:], bt[:] = k, p, t
    bp[n - 3] = -1
    with pytest.raises(TbeError):
        q.wait_batch(bk, bp, bt, 3 * n, bs, br)
    v2, t2 = q.export_state()
    assert np.array_equal(t2, tt) and np.array_equal(v2.view(np.uint64), v.view(np.uint64))
    for x in bufs:
        x.free()
    qref.close()
    aref.close()
