"""The token-bucket fold (k_fold_wide / k_fold_sparse) against the C restatement, bit for bit, on
bucket shapes chosen to land in every path: full single-chunk buckets (config B's),
buckets with rows of many requests, multi-chunk buckets, sparse buckets, a partial last
bucket, expiry deletions, zero and over-limit permits, one- and four-byte replies."""
import numpy as np
import pytest

from oracle import cref, trace

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000
ABSENT = np.iinfo(np.int64).min


def run(n_keys, cap, tokens, period, batches, narrow=True, p_choices=(1,), spread_us=10_000,
        seed=1, skew=0.0, ts_jitter=0):
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    eng = TokenBucketEngine(n_keys, cap, tokens, period, device=0, narrow=narrow)
    ref = cref.CTokenBucket(n_keys, cap, fill_rate(tokens, period))
    rng = np.random.default_rng(seed)
    outs = []
    for b, n in enumerate(batches):
        k = rng.integers(0, n_keys, n).astype(np.uint64)
        if skew:
            hot = rng.integers(0, n_keys, 4).astype(np.uint64)
            k = np.where(rng.random(n) < skew, hot[rng.integers(0, 4, n)], k)
        p = rng.choice(np.array(p_choices, np.int32), n)
        t = trace.batch_timestamps(b, n, spread_us)
        if ts_jitter:
            t = t + rng.integers(-ts_jitter, ts_jitter, n)
        g, r = eng.acquire_batch(k, p, t)
        g_ref, r_ref = ref.acquire_batch(k, p, t)
        bad = np.flatnonzero((g != g_ref) | (r != r_ref))
        assert bad.size == 0, (b, bad[:5], g[bad[:5]], r[bad[:5]], g_ref[bad[:5]], r_ref[bad[:5]])
        outs.append((g, r))
    v, t_us = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(t_us, t_ref)
    touched = t_ref != ABSENT
    assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
    return outs


@pytest.mark.parametrize("case", ["config_b_like", "small_rows", "busy_rows", "partial_last", "mixed_permits",
                                  "fast_refill_wide", "skew_hot", "jitter_expiry", "tail_long_run"])
def test_fold_shapes(engine_lib, gpu, case):
    if case == "config_b_like":      # R = 2048, ~1400 requests per bucket: all full
        run(3_000_000, 10, 1, 10_000_000, [1 << 21] * 3)
    elif case == "small_rows":       # R = 16, ~40 requests per bucket
        run(2_000, 5, 3, 10_000_000, [5_000] * 6, p_choices=(0, 1, 1, 2, 6))
    elif case == "busy_rows":        # R = 16, ~150 per bucket: rows of many requests
        run(3_000, 5, 3, 10_000_000, [28_000] * 4, p_choices=(1, 2))
    elif case == "partial_last":     # odd table: last bucket partial; a bucket of >2048
        run(1_000_003, 20, 50, 10_000_000, [700_000, 1_400_000, 700_000], p_choices=(1, 3))
    elif case == "mixed_permits":    # p = 0 always modifies; p > TokenLimit never grants
        run(500_000, 8, 4, 10_000_000, [400_000] * 4, p_choices=(0, 1, 2, 9, 3))
    elif case == "fast_refill_wide": # 4-byte replies (TokenLimit 1000), remaining spans 0..1000
        run(400_000, 1000, 40_000, 10_000_000, [350_000] * 3, narrow=False, p_choices=(1, 7, 50))
    elif case == "skew_hot":         # a few keys take 30%: their buckets go multi-chunk
        run(1_000_000, 10, 1, 10_000_000, [600_000] * 4, skew=0.3)
    elif case == "tail_long_run":    # 4 keys with ~60 requests each in config-B-like buckets:
        # after round 1 their runs exceed the tail walk's 32 (the rounds over the sorted list
        # take them) while every other bucket's tail is walked
        run(3_000_000, 10, 1, 10_000_000, [1 << 21] * 3, skew=240 / (1 << 21))
    elif case == "jitter_expiry":    # unsorted timestamps, TTL 3 s, batches 4 s apart
        run(300_000, 5, 2, 10_000_000, [250_000] * 4, spread_us=4_000_000, ts_jitter=900_000,
            p_choices=(0, 1, 3, 6))
