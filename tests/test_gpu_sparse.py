"""Sparse batches: a batch far smaller than the key space (2^14 to 2^23
requests over 1e8 keys) leaves most of the 48,829 buckets with a few requests each.  Those
go to k_fold_sparse -- one wave per bucket, the lanes of one key ballot-matched and walked
in arrival order by the key's first lane (TB:202-238) -- and the buckets of >= R/8 requests
to k_fold_wide through the dense-bucket list the bucket scan builds.  A sparse batch runs
no hot-key machinery: a Zipf batch's busiest keys fill dense buckets instead.  Every reply
and the table against the C restatement (oracle/tb_ref.c): uniform batches of every sparse
size, a skewed batch whose sparse buckets span several 64-request chunks with keys repeated
across chunks, dense buckets inside a sparse batch, Zipf batches, mixed permits, expiry,
and the unpacked (SoA) records."""
import os

import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))
T0 = 1_760_000_000_000_000
ABSENT = np.iinfo(np.int64).min


def _check_table(eng, ref):
    v, t = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(t, t_ref), np.flatnonzero(t != t_ref)[:10]
    touched = t_ref != ABSENT
    assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))


def _run(eng, ref, keys, permits, ts, tag):
    g, r = eng.acquire_batch(keys, permits, ts)
    g_ref, r_ref = ref.acquire_batch(keys, permits, ts, threads=THREADS)
    bad = np.flatnonzero((g != g_ref) | (r != r_ref))
    assert bad.size == 0, (tag, bad.size, bad[:5], keys[bad[:5]], g[bad[:5]], r[bad[:5]], g_ref[bad[:5]], r_ref[bad[:5]])


@pytest.mark.parametrize("logn", [14, 17, 20, 21, 22, 23])
def test_sparse_uniform_batches(engine_lib, gpu, logn):
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    n_keys, n = 100_000_000, 1 << logn
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n)
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    rng = np.random.default_rng(logn)
    for b in range(4):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.integers(0, 4, n).astype(np.int32)
        ts = (T0 + b * 400_000 + np.sort(rng.integers(0, 300_000, n))).astype(np.int64)
        _run(eng, ref, keys, permits, ts, (logn, b))
    _check_table(eng, ref)
    eng.close()


def test_small_sparse_batches_between_hot_batches(engine_lib, gpu):
    """sparse batches below 2^20 requests take no hot-key runs and leave the hot
    sets as they are (their busiest key fills one dense bucket, which k_fold_wide decides
    chunk by chunk); placed between dense 2^24 Zipf batches whose hot sets rotate, every
    reply and the table against the C restatement."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    n_keys = 100_000_000
    big = 1 << 24
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=big)
    assert eng.layout()["hot"]
    for m in (1 << 18, 1 << 19):
        assert eng.batch_format(m)["sparse"]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    rng = np.random.default_rng(23)
    perm = rng.permutation(1 << 20).astype(np.uint64) * 95 + 17   # Zipf ranks -> keys
    for b, m in enumerate([big, 1 << 19, 1 << 18, big, 1 << 19, big, big, 1 << 18]):
        ranks = np.minimum(rng.zipf(1.1, m), 1 << 20) - 1
        keys = perm[ranks]
        permits = rng.integers(0, 4, m).astype(np.int32)
        ts = (T0 + b * 2_000_000 + np.sort(rng.integers(0, 1_000_000, m))).astype(np.int64)
        _run(eng, ref, keys, permits, ts, (b, m))
    _check_table(eng, ref)
    eng.close()


def test_sparse_skewed_chunks_and_dense(engine_lib, gpu):
    """2^20 requests: 3% on 200 buckets (~157 requests each over 2048 rows: three chunks of
    64, keys repeated across them), 2% on 8 keys of one bucket (a dense bucket in a sparse
    batch: k_fold_wide via the list), 0.5% on 3 keys of 3 other buckets; timestamps over 30 s
    so that rows refill, lapse (TTL 10 s) and are re-granted."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    n_keys, n = 100_000_000, 1 << 20
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n)
    assert eng.layout()["passes"] == 2
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    rng = np.random.default_rng(7)
    for b in range(3):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        sel = rng.random(n)
        warm = sel < 0.03
        keys[warm] = (2048 * rng.integers(1000, 1200, warm.sum())
                      + rng.integers(0, 2048, warm.sum())).astype(np.uint64)
        hot = (sel >= 0.03) & (sel < 0.05)
        keys[hot] = (2048 * 777 + rng.integers(0, 8, hot.sum()) * 97).astype(np.uint64)
        few = (sel >= 0.05) & (sel < 0.055)
        keys[few] = np.array([2048 * 5 + 1, 2048 * 9000 + 2047, 2048 * 40000], np.uint64)[rng.integers(0, 3, few.sum())]
        permits = rng.integers(0, 5, n).astype(np.int32)
        ts = (T0 + b * 12_000_000 + np.sort(rng.integers(0, 10_000_000, n))).astype(np.int64)
        _run(eng, ref, keys, permits, ts, b)
    _check_table(eng, ref)
    eng.close()


def test_sparse_unpacked_records(engine_lib, gpu):
    """The SoA partition records (TBE_FLAG_NO_PACK) through the sparse fold."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    n_keys, n = 30_000_000, 1 << 18
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=n, pack=False)
    assert not eng.layout()["packed"]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    rng = np.random.default_rng(3)
    for b in range(3):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        keys[: n // 50] = rng.integers(0, 4096, n // 50).astype(np.uint64)   # two busier buckets
        rng.shuffle(keys)
        permits = rng.integers(0, 3, n).astype(np.int32)
        ts = (T0 + b * 2_000_000 + np.sort(rng.integers(0, 1_000_000, n))).astype(np.int64)
        _run(eng, ref, keys, permits, ts, b)
    _check_table(eng, ref)
    eng.close()


def test_sparse_zipf_batches(engine_lib, gpu):
    """Zipf(1.1) batches of 2^20 requests over 1e8 keys: sparse batches (fewer than R/8
    requests per bucket) that still run hot keys apart (hot runs are on from 2^20,
    TBE_HOT_SPARSE_MIN_LOG2: the busiest key, ~11% of a batch, ~115k requests, gets its own
    run), between dense 2^24 Zipf batches with hot runs."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    n_keys = 100_000_000
    big, n = 1 << 24, 1 << 20
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, max_batch=big)
    assert eng.layout()["hot"]
    assert eng.batch_format(n)["sparse"] and not eng.batch_format(big)["sparse"]
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    rng = np.random.default_rng(11)
    perm = rng.permutation(1 << 20).astype(np.uint64) * 95 + 17   # Zipf ranks -> keys
    for b, m in enumerate([big, n, n, big, n]):
        ranks = np.minimum(rng.zipf(1.1, m), 1 << 20) - 1
        keys = perm[ranks]
        permits = rng.integers(0, 4, m).astype(np.int32)
        ts = (T0 + b * 2_000_000 + np.sort(rng.integers(0, 1_000_000, m))).astype(np.int64)
        _run(eng, ref, keys, permits, ts, (b, m))
    _check_table(eng, ref)
    eng.close()
