"""GPU parity: the HIP engine (through the C ABI) against the CPU restatement, bit for bit.

Every test drives the same request trace through libtbe.so on cuda:0 and through the C
oracle (oracle/tb_ref.c), then compares granted/remaining per request and the full
bucket table (v bits and last-grant timestamps)."""
import ctypes

import zlib

import numpy as np
import pytest

from oracle import cref, trace
from oracle.semantics import new_t_of

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000
ABSENT = np.iinfo(np.int64).min


def make_pair(n_keys, token_limit, tokens_per_period, period_ticks, pack=True, **kw):
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    eng = TokenBucketEngine(n_keys, token_limit, tokens_per_period, period_ticks, device=0, pack=pack, **kw)
    ref = cref.CTokenBucket(n_keys, token_limit, fill_rate(tokens_per_period, period_ticks))
    return eng, ref


def assert_same_state(eng, ref):
    v, t = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(t, t_ref), f"t mismatch at {np.flatnonzero(t != t_ref)[:10]}"
    touched = t_ref != ABSENT
    bad = np.flatnonzero(v[touched].view(np.uint64) != v_ref[touched].view(np.uint64))
    assert bad.size == 0, f"v mismatch at {np.flatnonzero(touched)[bad[:10]]}"


def run_and_compare(eng, ref, keys, permits, ts):
    g, r = eng.acquire_batch(keys, permits, ts)
    g_ref, r_ref = ref.acquire_batch(keys, permits, ts)
    bad = np.flatnonzero((g != g_ref) | (r != r_ref))
    assert bad.size == 0, (f"{bad.size} mismatches, first at {bad[:5]}: gpu {g[bad[:5]]},{r[bad[:5]]} "
                           f"ref {g_ref[bad[:5]]},{r_ref[bad[:5]]}")
    return g, r


def test_kat_sequence(engine_lib, gpu):
    eng, ref = make_pair(64, 10, 1, 10_000_000)
    ps = np.array([1, 9, 1, 1, 0, 10, 11], dtype=np.int32)
    offs = [0, 500_000, 600_000, 1_000_000, 1_100_000, 5_000_000, 9_000_000]
    ts = np.array([S_US + o for o in offs], dtype=np.int64)
    keys = np.full(7, 42, dtype=np.uint64)
    g, r = run_and_compare(eng, ref, keys, ps, ts)
    assert g.tolist() == [1, 1, 0, 1, 1, 0, 0] and r.tolist() == [9, 0, 0, 0, 0, 4, 8]
    assert eng.query(42) == (float.fromhex("0x1.99998p-4"), new_t_of(S_US + 1_100_000))
    # the same KATs one request per batch (state carried across batches)
    eng2, _ = make_pair(64, 10, 1, 10_000_000)
    for i in range(7):
        g1, r1 = eng2.acquire_batch(keys[i:i + 1], ps[i:i + 1], ts[i:i + 1])
        assert (g1[0], r1[0]) == (g[i], r[i])


@pytest.mark.parametrize("n_keys,n,p_hi,interval,batches", [
    (1, 5000, 2, 2_000_000, 2),             # single key: every request collides
    (16, 4096, 3, 1_000_000, 3),            # r_bits floor, one bucket
    (1000, 2047, 1, 300_000, 3),            # just under one tile
    (1000, 2049, 4, 300_000, 3),            # just over one tile
    (10_000, 100_000, 3, 2_000_000, 3),     # config A shape
    (1 << 20, 300_000, 2, 10_000, 3),       # two LSD passes
    (3_000_017, 500_000, 1, 10_000, 2),     # odd table size, partial last bucket
])
@pytest.mark.parametrize("pack", [True, False], ids=["packed", "wide"])
def test_random_traces(engine_lib, gpu, n_keys, n, p_hi, interval, batches, pack):
    eng, ref = make_pair(n_keys, 10, 3, 10_000_000, pack=pack)
    assert eng.layout()["packed"] == pack
    for b in range(batches):
        k, p, t = trace.make_batch(0x5EED000B + n_keys, n_keys, b, n, interval, 0, p_hi)
        run_and_compare(eng, ref, k, p, t)
    assert_same_state(eng, ref)


@pytest.mark.parametrize("pack", [True, False], ids=["packed", "wide"])
def test_config_b_shape_small(engine_lib, gpu, pack):
    # Config B shape (100M keys, cap 10, 1 token/s, 10 ms batches), at 2^21 requests.
    eng, ref = make_pair(100_000_000, 10, 1, 10_000_000, pack=pack)
    lay = eng.layout()
    assert (lay["passes"], lay["r_bits"], lay["packed"], lay["hot"]) == (2, 11, pack, pack)
    for b in range(2):
        k, p, t = trace.make_batch(0x5EED000B, 100_000_000, b, 1 << 21, 10_000)
        g, _ = run_and_compare(eng, ref, k, p, t)
        assert g.mean() > 0.99  # fresh keys: almost all grant


def test_unsorted_timestamps_and_skew(engine_lib, gpu):
    rng = np.random.default_rng(5)
    n_keys, n = 500, 50_000
    eng, ref = make_pair(n_keys, 7, 2, 30_000_000)
    for b in range(3):
        k = rng.integers(0, n_keys, n, dtype=np.uint64)
        p = rng.integers(0, 9, n).astype(np.int32)             # includes p = 0 and p > cap
        t = (S_US + rng.integers(0, 20_000_000, n)).astype(np.int64)  # out of order
        run_and_compare(eng, ref, k, p, t)
    assert_same_state(eng, ref)


def test_fractional_rates(engine_lib, gpu):
    # rate 1/3 exercises the mul-then-add rounding that an FMA would break.
    rng = np.random.default_rng(9)
    eng, ref = make_pair(2000, 1, 1, 30_000_000)
    t = S_US
    for b in range(4):
        n = 40_000
        k = rng.integers(0, 2000, n, dtype=np.uint64)
        p = rng.integers(0, 2, n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 3_000_000, n))).astype(np.int64)
        t += 3_000_000
        run_and_compare(eng, ref, k, p, ts)
    assert_same_state(eng, ref)


def test_ttl_year_clamp_expiry(engine_lib, gpu):
    # 1 token per 10^7 s -> cap/rate = 1e8 s > 1 year: TTL clamps to 31536000 s.
    eng, ref = make_pair(4, 10, 1, 10**14)
    year = 31_536_000 * 1_000_000
    keys = np.zeros(3, dtype=np.uint64)
    g, r = run_and_compare(eng, ref, keys, np.array([10, 5, 5], np.int32),
                           np.array([S_US, S_US + year, S_US + year + 1000], np.int64))
    assert g.tolist() == [1, 0, 1] and r.tolist() == [0, 3, 5]


def test_empty_batch(engine_lib, gpu):
    eng, _ = make_pair(10, 5, 1, 10_000_000)
    g, r = eng.acquire_batch(np.zeros(0, np.uint64), np.zeros(0, np.int32), np.zeros(0, np.int64))
    assert g.size == 0 and r.size == 0


@pytest.mark.parametrize("bad", ["key", "permits", "ts"])
def test_invalid_batch_rejected_without_state_change(engine_lib, gpu, bad):
    from distributedratelimiting.redis_amd import TbeError
    eng, ref = make_pair(100, 5, 1, 10_000_000)
    k, p, t = trace.make_batch(3, 100, 0, 5000, 1_000_000)
    run_and_compare(eng, ref, k, p, t)
    k2, p2, t2 = trace.make_batch(3, 100, 1, 5000, 1_000_000)
    if bad == "key":
        k2[4321] = 100
    elif bad == "permits":
        p2[17] = -1
    else:
        t2[4999] = -5
    with pytest.raises(TbeError) as ei:
        eng.acquire_batch(k2, p2, t2)
    assert ei.value.status == 1
    assert_same_state(eng, ref)          # nothing applied
    k3, p3, t3 = trace.make_batch(3, 100, 2, 5000, 1_000_000)
    run_and_compare(eng, ref, k3, p3, t3)  # engine still usable


def test_device_api_and_generator(engine_lib, gpu):
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, fill_rate
    lib = _capi.load()
    lib.tbe_gen_batch_device.restype = ctypes.c_int
    lib.tbe_gen_batch_device.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_int32] * 2 + \
        [ctypes.c_int64] * 2 + [ctypes.c_void_p] * 4
    n_keys, n = 1_000_000, 1 << 18
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0)
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    dk = torch.empty(n, dtype=torch.int64, device=gpu)
    dp = torch.empty(n, dtype=torch.int32, device=gpu)
    dt = torch.empty(n, dtype=torch.int64, device=gpu)
    dg = torch.empty(n, dtype=torch.uint8, device=gpu)
    dr = torch.empty(n, dtype=torch.int32, device=gpu)
    for b in range(3):
        rc = lib.tbe_gen_batch_device(0x5EED000B, n_keys, b * n, n, 1, 4,
                                      trace.T0_US + b * 10_000, 10_000, dk.data_ptr(),
                                      dp.data_ptr(), dt.data_ptr(), None)
        assert rc == 0
        torch.cuda.synchronize()
        k, p, t = trace.make_batch(0x5EED000B, n_keys, b, n, 10_000, 1, 4)
        assert np.array_equal(dk.cpu().numpy().view(np.uint64), k)
        assert np.array_equal(dp.cpu().numpy(), p) and np.array_equal(dt.cpu().numpy(), t)
        eng.acquire_batch_device(dk, dp, dt, dg, dr)
        eng.synchronize()
        g_ref, r_ref = ref.acquire_batch(k, p, t)
        assert np.array_equal(dg.cpu().numpy(), g_ref)
        assert np.array_equal(dr.cpu().numpy(), r_ref)
    assert_same_state(eng, ref)


GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["tb_testapp_like", "tb_rate_third", "tb_tenth_second", "tb_skewed_clock",
                                  "tb_mixed_permits", "tb_year_ttl", "tb_fast_refill"])
@pytest.mark.parametrize("split", [1, 7])
def test_golden_reference_script(engine_lib, gpu, name, split):
    """GPU engine vs vectors recorded by executing the reference's Lua script
    (tests/golden/make_golden.py), one batch or split into `split` batches."""
    import os
    from distributedratelimiting.redis_amd import TokenBucketEngine
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    eng = TokenBucketEngine(int(g["n_keys"]), int(g["token_limit"]), int(g["tokens_per_period"]),
                            int(g["period_ticks"]), device=0)
    n = g["keys"].size
    cuts = np.linspace(0, n, split + 1).astype(int)
    gr, rem = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        x, y = eng.acquire_batch(g["keys"][a:b], g["permits"][a:b], g["ts_us"][a:b])
        gr.append(x); rem.append(y)
    assert np.array_equal(np.concatenate(gr), g["granted"])
    assert np.array_equal(np.concatenate(rem), g["remaining"])
    for k in range(int(g["n_keys"])):
        st = eng.query(k)
        if g["present"][k]:
            assert st == (g["v"][k], g["t"][k])
        else:
            assert st is None


def test_expired_key_deleted_even_when_denied(engine_lib, gpu):
    eng, ref = make_pair(3, 10, 1, 10**14)
    year = 31_536_000 * 1_000_000
    keys = np.zeros(3, np.uint64)
    g, r = run_and_compare(eng, ref, keys, np.array([10, 11, 3], np.int32),
                           np.array([S_US, S_US + year + 5_000, S_US + year - 5_000], np.int64))
    assert list(zip(g.tolist(), r.tolist())) == [(1, 0), (0, 10), (1, 7)]
    assert_same_state(eng, ref)


def test_packed_time_escape(engine_lib, gpu):
    """Packed records carry ts - (ts[0] - 2^(wb-1)) in wb bits; requests outside that
    window travel as escapes (their timestamp is re-read from the caller's array).
    TokenLimit 2^20 on 1000 keys leaves wb = 32 (+-35.8 min): spread the batch over +-3 h,
    with permits beyond TokenLimit (permit code clamped to TokenLimit + 1)."""
    rng = np.random.default_rng(77)
    cap = 1 << 20
    eng, ref = make_pair(1000, cap, 1000, 10_000_000)
    assert eng.layout()["packed"]
    hour = 3_600_000_000
    for b in range(3):
        n = 60_000
        k = rng.integers(0, 1000, n, dtype=np.uint64)
        p = rng.choice(np.array([0, 1, 7, cap - 1, cap, cap + 1, 2**31 - 1], np.int32), n)
        t = (S_US + b * hour + rng.integers(-3 * hour, 3 * hour, n)).astype(np.int64)
        run_and_compare(eng, ref, k, p, t)
    assert_same_state(eng, ref)
    # a batch whose first timestamp is 0 (window starts below zero), the rest far later
    t = np.full(5000, S_US + 10 * hour, np.int64)
    t[0] = 0
    run_and_compare(eng, ref, rng.integers(0, 1000, 5000, dtype=np.uint64),
                    np.ones(5000, np.int32), t)
    assert_same_state(eng, ref)


@pytest.mark.parametrize("pack", [True, False], ids=["packed", "wide"])
def test_hot_keys_speculative_rounds(engine_lib, gpu, pack):
    """Skewed traffic: a handful of keys take most requests, so chunks hold long same-key
    runs (mostly denies, settled by speculative rounds) mixed with rare grants and
    expiry deletions (p > TokenLimit on a lapsed key)."""
    rng = np.random.default_rng(11)
    n_keys = 50_000
    eng, ref = make_pair(n_keys, 5, 2, 10_000_000, pack=pack)
    for b in range(3):
        n = 200_000
        hot = rng.integers(0, n_keys, 8, dtype=np.uint64)
        k = np.where(rng.random(n) < 0.9, hot[rng.integers(0, 8, n)],
                     rng.integers(0, n_keys, n, dtype=np.uint64)).astype(np.uint64)
        p = rng.integers(0, 7, n).astype(np.int32)
        t = (S_US + b * 4_000_000 + np.sort(rng.integers(0, 4_000_000, n))).astype(np.int64)
        run_and_compare(eng, ref, k, p, t)
    assert_same_state(eng, ref)


@pytest.mark.parametrize("hot", [True, False], ids=["hot_runs", "no_hot"])
@pytest.mark.parametrize("cap,tokens,period", [(10, 1, 10_000_000), (100, 5000, 10_000_000)],
                         ids=["throttled", "fast_refill"])
def test_zipf_hot_runs(engine_lib, gpu, hot, cap, tokens, period):
    """Config C shape at test size: Zipf(1.1) keys, so the top keys take thousands of
    requests per batch and (from the second batch on) get runs of their own.  Throttled:
    hot runs are mostly denies (pass-through segments); fast refill: hot keys keep
    granting (segments decided serially in the chain)."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate, workloads
    n_keys, n = 1_000_000, 1 << 20
    eng = TokenBucketEngine(n_keys, cap, tokens, period, device=0, hot=hot)
    assert eng.layout()["hot"] == hot
    ref = cref.CTokenBucket(n_keys, cap, fill_rate(tokens, period))
    zs = workloads.ZipfSampler(n_keys, 1.1)
    rng = np.random.default_rng(3)
    for b in range(4):
        k = workloads.zipf_keys(0x5EED000C, n_keys, b * n, n, sampler=zs)
        p = np.where(rng.random(n) < 0.97, 1, rng.integers(0, cap + 3, n)).astype(np.int32)
        t = workloads.batch_timestamps(b, n, 10_000, trace.T0_US)
        run_and_compare(eng, ref, k, p, t)
    assert_same_state(eng, ref)


def test_hot_runs_unsorted_times_and_expiry(engine_lib, gpu):
    """Hot keys with unsorted timestamps spread over several TTLs (cap 5 at 2 tokens/s:
    TTL 3 s), permits 0..7 (p = 0 always modifies; p > 5 only ever deletes a lapsed
    key), and a hot set that changes from batch to batch."""
    rng = np.random.default_rng(21)
    n_keys = 3000                     # 188 ordinary buckets of 16 keys: room for 68 hot runs
    eng, ref = make_pair(n_keys, 5, 2, 10_000_000)
    assert eng.layout()["hot"]
    for b in range(5):
        n = 120_000
        hot = rng.integers(0, n_keys, 6, dtype=np.uint64)
        k = np.where(rng.random(n) < 0.8, hot[rng.integers(0, 6, n)],
                     rng.integers(0, n_keys, n, dtype=np.uint64)).astype(np.uint64)
        p = rng.integers(0, 8, n).astype(np.int32)
        t = (S_US + b * 9_000_000 + rng.integers(0, 9_000_000, n)).astype(np.int64)
        run_and_compare(eng, ref, k, p, t)
        assert_same_state(eng, ref)


def test_single_hot_key_many_segments(engine_lib, gpu):
    """One key takes a whole 300k-request batch (37 run segments) twice in a row; the
    refill lets it grant every ~1000 requests, so some segments pass through and others
    are decided in the chain."""
    eng, ref = make_pair(64, 3, 1, 10_000_000)
    n = 300_000
    for b in range(3):
        k = np.full(n, 17, np.uint64)
        t = (S_US + b * 300_000_000 + np.arange(n, dtype=np.int64) * 1000).astype(np.int64)
        run_and_compare(eng, ref, k, np.ones(n, np.int32), t)
    assert_same_state(eng, ref)


@pytest.mark.parametrize("narrow,cap", [(True, 127), (False, 10), (True, 1000)],
                         ids=["narrow_cap127", "wide_forced", "wide_cap1000"])
def test_reply_width(engine_lib, gpu, narrow, cap):
    """One-byte replies (TokenLimit <= 127) and four-byte ones (forced, or TokenLimit too
    large) through the fold, the hot-key runs and the un-partition passes, on Zipf traffic
    with a fast refill so remaining values span 0..TokenLimit."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate, workloads
    n_keys, n = 500_000, 1 << 19
    tokens = cap * 50
    eng = TokenBucketEngine(n_keys, cap, tokens, 10_000_000, device=0, narrow=narrow)
    assert eng.layout()["narrow"] == (narrow and cap <= 127)
    ref = cref.CTokenBucket(n_keys, cap, fill_rate(tokens, 10_000_000))
    zs = workloads.ZipfSampler(n_keys, 1.1)
    rng = np.random.default_rng(cap)
    for b in range(4):
        k = workloads.zipf_keys(0x5EED0007, n_keys, b * n, n, sampler=zs)
        p = rng.integers(0, 4, n).astype(np.int32)
        t = workloads.batch_timestamps(b, n, 10_000, trace.T0_US)
        g, r = run_and_compare(eng, ref, k, p, t)
    assert r.max() == cap or r.max() >= cap - 3
    assert_same_state(eng, ref)


def test_snapshot_restore(engine_lib, gpu):
    """Snapshot/restore of the bucket hashes (tbe_export_state -> tbe_import_state into a
    fresh engine): the restored engine continues the trace exactly like the original and
    the oracle, including absent keys and a partial-range restore."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, TbeError
    n_keys, n = 50_000, 200_000
    eng, ref = make_pair(n_keys, 10, 3, 10_000_000)
    for b in range(2):
        k, p, t = trace.make_batch(0x5EED0009, n_keys, b, n, 700_000, 1, 3)
        run_and_compare(eng, ref, k, p, t)
    v, t_us = eng.export_state()
    assert (t_us == ABSENT).any() and (t_us != ABSENT).any()
    fresh = TokenBucketEngine(n_keys, 10, 3, 10_000_000, device=0)
    fresh.import_state(v[:1000], t_us[:1000])                  # two ranges
    fresh.import_state(v[1000:], t_us[1000:], first=1000)
    for b in range(2, 4):
        k, p, t = trace.make_batch(0x5EED0009, n_keys, b, n, 700_000, 1, 3)
        g1, r1 = run_and_compare(eng, ref, k, p, t)
        g2, r2 = fresh.acquire_batch(k, p, t)
        assert np.array_equal(g1, g2) and np.array_equal(r1, r2)
    assert_same_state(fresh, ref)
    with pytest.raises(TbeError):
        fresh.import_state(v[:10], t_us[:10], first=n_keys - 5)


def test_hot_key_cools_down(engine_lib, gpu):
    """A key hot for a few batches (its row written by the hot-key chain with ordinary
    stores) then cold again (its row read back by the fold's streaming slice loads): the
    fold must see the chain's last write."""
    n_keys, n, hot_key = 100_000, 200_000, 4242
    eng, ref = make_pair(n_keys, 50, 5000, 10_000_000)
    rng = np.random.default_rng(11)
    for b in range(8):
        k = rng.integers(0, n_keys, n).astype(np.uint64)
        m = 5000 if b < 3 else 10
        k[rng.choice(n, m, replace=False)] = hot_key
        p = rng.integers(1, 4, n).astype(np.int32)
        t = trace.batch_timestamps(b, n, 10_000)
        run_and_compare(eng, ref, k, p, t)
        assert_same_state(eng, ref)


def test_config_struct_size_versions(engine_lib, gpu):
    """tbe_create accepts the first published tbe_config layout (struct_size 56, without
    zero_wait_slots/reserved) and reads the missing fields as 0; smaller sizes are EINVAL."""
    import ctypes
    from distributedratelimiting.redis_amd import _capi
    lib = _capi.load()
    cfg = _capi.make_config(1000, 5, 1, 10_000_000, device=0)
    for size, ok in ((ctypes.sizeof(_capi.TbeConfig), True), (56, True), (55, False), (0, False)):
        cfg.struct_size = size
        h = ctypes.c_void_p()
        st = lib.tbe_create(ctypes.byref(cfg), ctypes.byref(h))
        assert (st == _capi.TBE_OK) == ok, (size, st)
        if ok:
            k = np.arange(10, dtype=np.uint64)
            g = np.empty(10, np.uint8)
            r = np.empty(10, np.int32)
            t = np.full(10, 1_760_000_000_000_000, np.int64)
            p = np.ones(10, np.int32)
            assert lib.tbe_acquire_batch(h, k.ctypes.data, p.ctypes.data, t.ctypes.data, 10, g.ctypes.data,
                                         r.ctypes.data) == _capi.TBE_OK
            assert g.all() and (r == 4).all()
            lib.tbe_destroy(h)
        else:
            assert st == _capi.TBE_EINVAL


@pytest.mark.parametrize("n_keys,n,batches", [(3_000_000, 2_000_000, 3), (600_000, 50_000, 4),
                                               (1 << 24, 300_000, 2), (70_000, 1_200_000, 3)])
def test_two_pass_partition_shapes(engine_lib, gpu, n_keys, n, batches):
    """Two LSD passes over many tiles, one partial tile, and tiles that straddle the first
    pass's digit boundaries (small key spaces), mixed permits: replies and table against
    the C restatement."""
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    eng = TokenBucketEngine(n_keys, 6, 2, 10_000_000, device=0)
    assert eng.layout()["passes"] >= 2
    ref = cref.CTokenBucket(n_keys, 6, fill_rate(2, 10_000_000))
    for b in range(batches):
        keys, permits, ts = trace.make_batch(0x100C + n, n_keys, b, n, 900_000, 0, 3)
        g, r = eng.acquire_batch(keys, permits, ts)
        g_ref, r_ref = ref.acquire_batch(keys, permits, ts)
        assert np.array_equal(g, g_ref) and np.array_equal(r, r_ref), b
    v, t = eng.export_state()
    v_ref, t_ref = ref.export_state()
    touched = t_ref != np.iinfo(np.int64).min
    assert np.array_equal(t, t_ref)
    assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
    eng.close()
    ref.close()


@pytest.mark.parametrize("case", ["two_pass", "two_pass_escape", "two_pass_hot", "three_pass", "sparse"])
@pytest.mark.parametrize("fold,digits,rerank", [(True, True, False), (False, True, False), (True, False, False),
                                                (True, True, True)],
                         ids=["fold_records", "unscatter_all", "hist_records", "rerank"])
def test_fold_records_layouts(engine_lib, gpu, case, fold, digits, rerank):
    """Fold records (the last partition pass carries each request's position in its input;
    the fold, the sparse fold and the hot runs reply straight there), against
    TBE_FLAG_UNSCATTER_ALL and the C restatement:
    two passes; timestamps spread over hours (fold records escape to the previous pass's
    record, itself escaping to the caller's array); hot-key runs; three passes (> 2^27
    keys: 65536 reply regions); a sparse batch (the density gate sends its buckets to
    k_fold_sparse).  rerank: the final un-partition re-ranks pass 0's tiles (k_unrank) instead of
    gathering through pass 0's permutation.  hist_records: the second pass's histogram
    reads the first pass's records instead of the digit stream (k_hist_dig), whose tiles
    here lie inside one pass-0 digit, straddle a few or (sparse) span many."""
    rng = np.random.default_rng(zlib.crc32(case.encode()) % 1000)
    n_keys = {"three_pass": 140_000_000, "sparse": 100_000_000}.get(case, 3_000_000)
    n = {"sparse": 1 << 16, "three_pass": 300_000}.get(case, 400_000)
    # three passes (> 2^27 keys: a 28-bit key field) pack only with a 3-bit permit code
    eng, ref = make_pair(n_keys, 6 if case == "three_pass" else 10, 3, 10_000_000, fold_records=fold,
                         digit_stream=digits, rerank=rerank)
    lay = eng.layout()
    assert lay["fold_records"] == fold and lay["passes"] == (3 if case == "three_pass" else 2)
    assert lay["digit_stream"] == (digits and case != "three_pass")
    assert lay["rerank"] == (fold and rerank)
    hot = rng.integers(0, n_keys, 20).astype(np.uint64)
    t = S_US
    for b in range(4 if case == "two_pass_hot" else 2):
        k = rng.integers(0, n_keys, n).astype(np.uint64)
        if case == "two_pass_hot":
            sel = rng.random(n) < 0.8
            k[sel] = hot[rng.integers(0, 20, int(sel.sum()))]
        p = rng.integers(0, 4, n).astype(np.int32)
        span = 3 * 3_600_000_000 if case == "two_pass_escape" else 10_000
        ts = (t + np.sort(rng.integers(0, span, n))).astype(np.int64)
        if case == "two_pass_escape":
            rng.shuffle(ts[: n // 2])       # out of order too
        t = int(ts.max()) + 1
        run_and_compare(eng, ref, k, p, ts)
    if case != "three_pass":
        assert_same_state(eng, ref)
    else:   # 2.2 GB tables: the rows the batches touched
        touched = np.unique(k)
        v, tt = eng.export_state()
        v_ref, t_ref = ref.export_state()
        assert np.array_equal(tt[touched], t_ref[touched])
        assert np.array_equal(v[touched].view(np.uint64), v_ref[touched].view(np.uint64))
        assert np.array_equal(tt != ABSENT, t_ref != ABSENT)
