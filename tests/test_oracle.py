"""CPU tests of the oracle itself: KATs, two independent restatements agreeing bit for
bit, generator equality, and properties of the reference semantics."""
import math
import subprocess

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from oracle import cref, trace
from oracle.semantics import (TokenBucketConfig, TokenBucketTable, fill_rate_per_second,
                              lua_max, lua_min, new_t_of, tb_ttl_seconds)

S_US = 1_760_572_800 * 1_000_000


def kat_sequence():
    # cap 10, rate 1.0, one key.
    return [  # (permits, ts offset us, granted, remaining, state v after or None=unchanged)
        (1, 0, True, 9, 9.0),
        (9, 500_000, True, 0, 0.5),
        (1, 600_000, False, 0, None),
        (1, 1_000_000, True, 0, 0.0),
        (0, 1_100_000, True, 0, float.fromhex("0x1.99998p-4")),
        (10, 5_000_000, False, 4, None),
        (11, 9_000_000, False, 8, None),
    ]


def test_kat_python():
    tb = TokenBucketTable(TokenBucketConfig(10, 1.0))
    last = None
    for p, dt, g, r, v in kat_sequence():
        assert tb.acquire(42, p, S_US + dt) == (g, r)
        st_ = tb.query(42)
        if v is not None:
            assert st_[0] == v and st_[1] == new_t_of(S_US + dt)
            last = st_
        else:
            assert st_ == last


def test_kat_denied_refill_value():
    # KAT 3: x = 0x1.33333p-1 (dt quantised by ulp(t) ~ 2.4e-7 s at 1.76e9 s)
    tb = TokenBucketTable(TokenBucketConfig(10, 1.0))
    tb.acquire(1, 1, S_US)
    tb.acquire(1, 9, S_US + 500_000)
    _, x, _ = tb.refill(1, S_US + 600_000)
    assert x == float.fromhex("0x1.33333p-1")


def test_kat_c():
    c = cref.CTokenBucket(64, 10, 1.0)
    ps = np.array([k[0] for k in kat_sequence()], dtype=np.int32)
    ts = np.array([S_US + k[1] for k in kat_sequence()], dtype=np.int64)
    keys = np.full(len(ps), 42, dtype=np.uint64)
    g, r = c.acquire_batch(keys, ps, ts)
    assert g.tolist() == [1 if k[2] else 0 for k in kat_sequence()]
    assert r.tolist() == [k[3] for k in kat_sequence()]
    assert c.query(42)[0] == float.fromhex("0x1.99998p-4")


def test_fill_rate_and_ttl():
    assert fill_rate_per_second(10, 10_000_000) == 10.0
    assert fill_rate_per_second(1, 1_000_000) == 10.0          # TestApp 0.1 s period
    assert cref.load().tbr_fill_rate(3, 70_000_000) == fill_rate_per_second(3, 70_000_000)
    assert tb_ttl_seconds(10, 1.0) == 10
    assert tb_ttl_seconds(1, 1000.0) == 1                       # lower clamp
    assert tb_ttl_seconds(10, 1e-9) == 31_536_000               # upper clamp
    assert math.isinf(fill_rate_per_second(1, 0))
    with pytest.raises(ValueError):
        TokenBucketConfig.from_options(10, 1, 0)                 # "∞" script, Appendix B
    with pytest.raises(ValueError):
        TokenBucketConfig.from_options(0, 1, 10_000_000)


def test_lua_minmax_argument_order():
    assert math.copysign(1.0, lua_max(0.0, -0.0)) == 1.0
    assert math.copysign(1.0, lua_max(-0.0, 0.0)) == -1.0
    assert lua_max(0.0, float("nan")) == 0.0
    assert math.isnan(lua_min(float("nan"), 1.0))


def test_generators_identical(oracle_lib):
    for K, b, n in [(10_000, 0, 1000), (100_000_000, 5, 4096), (3, 2, 777)]:
        a = trace.make_batch(0x5EED000B, K, b, n, 10_000, 1, 4)
        c = cref.gen_batch(0x5EED000B, K, b, n, 10_000, 1, 4)
        for x, y in zip(a, c):
            assert np.array_equal(x, y)
        assert a[0].max() < K and a[1].min() >= 1 and a[1].max() <= 4
        assert np.all(np.diff(a[2]) >= 0)


@pytest.mark.parametrize("n_keys,n,p_hi,interval", [
    (1, 3000, 3, 1_000_000), (16, 5000, 2, 300_000), (1000, 20000, 4, 2_000_000),
    (10_000, 30000, 1, 2_000_000)])
def test_python_vs_c(oracle_lib, n_keys, n, p_hi, interval):
    cfg = TokenBucketConfig.from_options(20, 10, 10_000_000)
    py = TokenBucketTable(cfg)
    c = cref.CTokenBucket(n_keys, cfg.token_limit, cfg.fill_rate)
    for b in range(3):
        k, p, t = trace.make_batch(7 + b, n_keys, b, n, interval, 0, p_hi)
        g1, r1 = py.acquire_batch(k, p, t)
        g2, r2 = c.acquire_batch(k, p, t)
        assert np.array_equal(np.array(g1, dtype=np.uint8), g2)
        assert np.array_equal(np.array(r1, dtype=np.int32), r2)
    v, tt = c.export_state()
    for key in range(n_keys):
        s = py.state.get(key)
        if s is None:
            assert tt[key] == np.iinfo(np.int64).min
        else:
            assert s.t_us == tt[key] and s.v == v[key]


def test_c_multithreaded_matches_serial(oracle_lib):
    k, p, t = trace.make_batch(11, 5000, 0, 200_000, 1_000_000, 1, 3)
    a = cref.CTokenBucket(5000, 7, 3.0)
    b = cref.CTokenBucket(5000, 7, 3.0)
    g1, r1 = a.acquire_batch(k, p, t, threads=1)
    g2, r2 = b.acquire_batch(k, p, t, threads=4)
    assert np.array_equal(g1, g2) and np.array_equal(r1, r2)


def test_c_oracle_has_no_fma(oracle_lib):
    dis = subprocess.run(["objdump", "-d", oracle_lib], capture_output=True, text=True).stdout
    assert "vfmadd" not in dis and "vfmsub" not in dis


@settings(max_examples=200, deadline=None)
@given(cap=st.integers(1, 1000), tokens=st.integers(1, 1000),
       ticks=st.integers(1, 10**9),
       reqs=st.lists(st.tuples(st.integers(0, 5), st.integers(0, 1200), st.integers(0, 3_000_000)),
                     min_size=1, max_size=60))
def test_properties(cap, tokens, ticks, reqs):
    cfg = TokenBucketConfig.from_options(cap, tokens, ticks)
    tb = TokenBucketTable(cfg)
    c = cref.CTokenBucket(6, cap, cfg.fill_rate)
    ts = S_US
    keys, ps, tss, out = [], [], [], []
    for key, p, dt in reqs:
        ts += dt
        before = tb.state.get(key)
        before = None if before is None else (before.v, before.t_us)
        g, r = tb.acquire(key, p, ts)
        after = tb.state.get(key)
        after = None if after is None else (after.v, after.t_us)
        assert 0 <= r <= cap
        if p == 0:
            assert g                                 # x >= 0 always
        if p > cap:
            assert not g                             # x <= cap always
        if not g:
            assert after == before or (before is not None and after is None)  # deny writes nothing
        keys.append(key); ps.append(p); tss.append(ts); out.append((int(g), r))
    g2, r2 = c.acquire_batch(np.array(keys), np.array(ps), np.array(tss))
    assert [(int(a), int(b)) for a, b in zip(g2, r2)] == out


def test_expiry_one_year_clamp():
    # cap/rate = 1e8 s > 1 year: the key lapses 31536000 s after its last grant and the
    # next request sees a full bucket (TB:232-235 + Redis passive expiry).
    cfg = TokenBucketConfig(10, 1e-7)
    tb = TokenBucketTable(cfg)
    assert tb.acquire(0, 10, S_US) == (True, 0)
    year_us = 31_536_000 * 1_000_000
    assert tb.acquire(0, 5, S_US + year_us) == (False, 3)          # not yet lapsed (== when)
    assert tb.acquire(0, 5, S_US + year_us + 1000) == (True, 5)   # lapsed: default {cap, now}
    c = cref.CTokenBucket(1, 10, 1e-7)
    g, r = c.acquire_batch(np.zeros(3, np.uint64), np.array([10, 5, 5]),
                           np.array([S_US, S_US + year_us, S_US + year_us + 1000]))
    assert g.tolist() == [1, 0, 1] and r.tolist() == [0, 3, 5]


def test_clock_skew_backwards():
    # TB:217-218: a timestamp earlier than the stored t refills nothing, and a grant
    # then stores the earlier t.
    tb = TokenBucketTable(TokenBucketConfig(5, 1.0))
    assert tb.acquire(3, 5, S_US + 10_000_000) == (True, 0)
    assert tb.acquire(3, 0, S_US) == (True, 0)
    assert tb.query(3) == (0.0, new_t_of(S_US))
    assert tb.acquire(3, 1, S_US + 1_000_000) == (True, 0)   # refill from the earlier t


def test_expired_key_deleted_even_when_denied():
    # Passive expiry deletes the key at the HGETALL (TB:210) even if the script then
    # denies (p > cap): a later request with an EARLIER timestamp must see it absent.
    cfg = TokenBucketConfig(10, 1e-7)
    year = 31_536_000 * 1_000_000
    seq = [(0, 10, S_US), (0, 11, S_US + year + 5_000), (0, 3, S_US + year - 5_000)]
    tb = TokenBucketTable(cfg)
    out = [tb.acquire(k, p, t) for k, p, t in seq]
    assert out == [(True, 0), (False, 10), (True, 7)]
    assert tb.query(0) == (7.0, new_t_of(S_US + year - 5_000))
    c = cref.CTokenBucket(1, 10, 1e-7)
    g, r = c.acquire_batch(np.zeros(3, np.uint64), np.array([s[1] for s in seq]),
                           np.array([s[2] for s in seq]))
    assert list(zip(g.tolist(), r.tolist())) == [(1, 0), (0, 10), (1, 7)]
