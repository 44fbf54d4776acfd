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
