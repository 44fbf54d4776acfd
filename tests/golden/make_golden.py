#!/usr/bin/env python3
"""Generate golden vectors by executing the REFERENCE's own Lua scripts.

    python tests/golden/make_golden.py      (needs /root/reference; run in the build container)

For each case the script text is pulled out of the reference C# source
(TokenBucket/RedisTokenBucketRateLimiter.cs GetAcquireLuaScript, TB:176-239;
ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs GetAcquireLuaScript,
A:216-271), interpolated as C# would, and run by oracle/lua_replay.py against a mock
Redis with injected TIME.  Only inputs and outputs are written (``*.npz``, no
pickles, plus ``manifest.json``); no reference source text is stored.  The GPU box
never runs this script: it only reads the committed fixtures.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.lua_replay import ReferenceApproxSync, ReferenceTokenBucket  # noqa: E402
from oracle.semantics import fill_rate_per_second  # noqa: E402

S_US = 1_760_572_800 * 1_000_000

TB_CASES = [  # (name, TokenLimit, TokensPerPeriod, period ticks, n_keys, n, style, mean gap us)
    ("tb_testapp_like", 20, 10, 10_000_000, 6, 3000, "monotone", 4_000),      # config A shape
    ("tb_rate_third", 10, 1, 30_000_000, 25, 3000, "monotone", 40_000),      # rate 1/3 (FMA-sensitive)
    ("tb_tenth_second", 100, 1, 1_000_000, 3, 2000, "monotone", 30_000),     # TestApp period 0.1 s
    ("tb_skewed_clock", 7, 3, 20_000_000, 30, 3000, "shuffled", 40_000),     # non-monotone TIME
    ("tb_mixed_permits", 5, 2, 10_000_000, 12, 3000, "bursty", 400_000),     # p in 0..cap+2
    ("tb_year_ttl", 10, 1, 10**14, 6, 400, "sparse_years", 0),               # TTL clamp, expiry
    ("tb_fast_refill", 3, 1000, 10_000_000, 2, 2000, "monotone", 1_000),     # TTL floor 1 s
]


def tb_trace(rng, n_keys, n, style, cap, gap):
    keys = rng.integers(0, n_keys, n).astype(np.uint64)
    if style in ("bursty", "sparse_years"):
        permits = rng.integers(0, cap + 3, n).astype(np.int32)
    else:
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
    if style == "monotone":
        ts = S_US + np.cumsum(rng.integers(0, 2 * gap, n))
    elif style == "shuffled":
        ts = S_US + np.cumsum(rng.integers(0, 2 * gap, n))
        idx = rng.permutation(n)[: n // 4]
        ts[idx] -= rng.integers(0, 3_000_000, idx.size)      # clock steps backwards
    elif style == "bursty":
        ts = S_US + np.repeat(np.cumsum(rng.integers(0, 2 * gap, n // 20 + 1)), 20)[:n]
    else:  # sparse_years: gaps around the 1-year TTL boundary
        year = 31_536_000 * 1_000_000
        gaps = rng.choice([0, 1_000, year - 2_000, year, year + 1_000, 5_000_000], n)
        ts = S_US + np.cumsum(gaps)
    return keys, permits, ts.astype(np.int64)


def make_tb(out_dir, manifest):
    for i, (name, cap, tokens, ticks, n_keys, n, style, gap) in enumerate(TB_CASES):
        rng = np.random.default_rng(1000 + i)
        rate = fill_rate_per_second(tokens, ticks)
        keys, permits, ts = tb_trace(rng, n_keys, n, style, cap, gap)
        ref = ReferenceTokenBucket(cap, rate)
        granted = np.empty(n, np.uint8)
        remaining = np.empty(n, np.int32)
        for j in range(n):
            g, r = ref.acquire(int(keys[j]), int(permits[j]), int(ts[j]))
            granted[j], remaining[j] = g, r
        # final Redis hash state (after passive expiry at the last timestamp is NOT applied:
        # the hash as stored)
        present = np.zeros(n_keys, np.uint8)
        v = np.zeros(n_keys, np.float64)
        t = np.zeros(n_keys, np.float64)
        for k in range(n_keys):
            st = ref.state(k)
            if st is not None:
                present[k], v[k], t[k] = 1, st[0], st[1]
        np.savez(os.path.join(out_dir, f"{name}.npz"), keys=keys, permits=permits, ts_us=ts,
                 granted=granted, remaining=remaining, present=present, v=v, t=t,
                 token_limit=np.int32(cap), tokens_per_period=np.int32(tokens),
                 period_ticks=np.int64(ticks), fill_rate=np.float64(rate), n_keys=np.int64(n_keys))
        manifest[name] = {"kind": "token_bucket", "script": "TB:181-238 GetAcquireLuaScript",
                          "token_limit": cap, "tokens_per_period": tokens, "period_ticks": ticks,
                          "fill_rate_hex": rate.hex(), "n_keys": n_keys, "n": n, "style": style,
                          "grant_rate": float(granted.mean())}
        print(f"{name}: {n} requests, grant rate {granted.mean():.3f}")


def make_approx(out_dir, manifest):
    # Sync script calls: (bucket, LocalCount, TIME) -> (global score, period, period string).
    cases = [("approx_one_client", 10, 10_000_000, 1, 60), ("approx_eight_clients", 100, 1_000_000, 8, 60),
             ("approx_slow_decay", 5, 70_000_000, 3, 80)]
    for i, (name, tokens, ticks, clients, rounds) in enumerate(cases):
        rng = np.random.default_rng(2000 + i)
        rate = fill_rate_per_second(tokens, ticks)
        period_us = ticks // 10
        ref = ReferenceApproxSync(rate)
        counts, tss, glob, per, per_str = [], [], [], [], []
        t = S_US
        for r in range(rounds):
            for c in range(clients):
                ts = t + (c * period_us) // clients + int(rng.integers(0, 2_000))
                if rng.random() < 0.1:
                    ts -= int(rng.integers(0, 3 * period_us))              # skewed clock
                cnt = int(rng.integers(0, 3 * tokens + 1))
                g, p, ps = ref.sync("approx:default", cnt, ts)
                counts.append(cnt); tss.append(ts); glob.append(g); per.append(p); per_str.append(ps)
            t += period_us
        st = ref.state("approx:default")
        np.savez(os.path.join(out_dir, f"{name}.npz"), counts=np.array(counts, np.int32),
                 ts_us=np.array(tss, np.int64), global_score=np.array(glob, np.int64),
                 period=np.array(per, np.float64),
                 period_str=np.array(per_str, dtype="U32"),
                 final_v=np.float64(st["v"]), final_p=np.float64(st["p"]), final_t=np.float64(st["t"]),
                 decay_rate=np.float64(rate), tokens_per_period=np.int32(tokens),
                 period_ticks=np.int64(ticks), clients=np.int32(clients))
        manifest[name] = {"kind": "approximate_sync", "script": "A:221-270 GetAcquireLuaScript",
                          "tokens_per_period": tokens, "period_ticks": ticks, "clients": clients,
                          "calls": len(counts)}
        print(f"{name}: {len(counts)} sync calls")


def main():
    out_dir = HERE
    manifest = {"generator": "tests/golden/make_golden.py",
                "engine": "oracle/lua_replay.py executing the reference's Lua script text",
                "cases": {}}
    make_tb(out_dir, manifest["cases"])
    make_approx(out_dir, manifest["cases"])
    with open(os.path.join(out_dir, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
