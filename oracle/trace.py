"""Seeded, counter-based request-trace generator (TEST INFRASTRUCTURE).

The same generator exists three times and must produce identical bytes:
  * here (numpy, used by tests and fixture scripts),
  * ``oracle/tb_ref.c`` (``tbr_gen_*``, used by the CPU baseline),
  * ``distributedratelimiting.redis_amd/csrc/tbe_gen.hip`` (device-side generation
    for bench.py, so PCIe never sits in the timed region).

Request ``g`` (global request counter = batch * n + i) of stream ``s`` draws
``r = mix64(seed ^ STREAM[s] + g * GAMMA)`` where ``mix64`` is the splitmix64
finaliser.  Keys are ``((r >> 32) * n_keys) >> 32`` (uniform on [0, n_keys),
n_keys < 2**32).  Timestamps follow SURVEY.md §8(d): batch ``b`` spans
``interval_us`` microseconds starting at ``t0_us + b * interval_us`` and request
``i`` of ``n`` gets ``t0_us + b*interval_us + (i*interval_us)//n`` (non-decreasing).

The reference has no trace format or generator (it has no tests at all,
SURVEY.md §4); this one is the build's own.
"""
from __future__ import annotations

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1

STREAM_KEY = 0x0000000000000000
STREAM_PERMITS = 0xA5A5A5A5A5A5A5A5
STREAM_ZIPF = 0x3C3C3C3C3C3C3C3C

T0_US = 1_760_000_000_000_000  # 2025-10-09T09:46:40Z, SURVEY.md §8(d) config A


def mix64_scalar(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * M1) & MASK64
    z = ((z ^ (z >> 27)) * M2) & MASK64
    return z ^ (z >> 31)


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(M1)
        z ^= z >> np.uint64(27)
        z *= np.uint64(M2)
        z ^= z >> np.uint64(31)
    return z


def stream(seed: int, stream_id: int, g0: int, n: int) -> np.ndarray:
    """r[g] for g in [g0, g0+n): mix64((seed ^ stream_id) + g * GAMMA)."""
    base = np.uint64((seed ^ stream_id) & MASK64)
    g = np.arange(g0, g0 + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = base + g * np.uint64(GAMMA)
    return mix64(z)


def uniform_keys(seed: int, n_keys: int, g0: int, n: int) -> np.ndarray:
    assert 0 < n_keys < (1 << 32)
    r = stream(seed, STREAM_KEY, g0, n)
    return ((r >> np.uint64(32)) * np.uint64(n_keys)) >> np.uint64(32)


def permits(seed: int, g0: int, n: int, lo: int = 1, hi: int = 1) -> np.ndarray:
    """Permits uniform on {lo..hi} (inclusive); constant when lo == hi."""
    if lo == hi:
        return np.full(n, lo, dtype=np.int32)
    span = hi - lo + 1
    r = stream(seed, STREAM_PERMITS, g0, n)
    return (lo + (((r >> np.uint64(32)) * np.uint64(span)) >> np.uint64(32))).astype(np.int32)


def batch_timestamps(batch: int, n: int, interval_us: int, t0_us: int = T0_US) -> np.ndarray:
    i = np.arange(n, dtype=np.int64)
    return t0_us + batch * interval_us + (i * interval_us) // n


def make_batch(seed: int, n_keys: int, batch: int, n: int, interval_us: int,
               p_lo: int = 1, p_hi: int = 1, t0_us: int = T0_US):
    """(keys u64, permits i32, ts_us i64) for batch ``batch`` of a config-B style trace."""
    g0 = batch * n
    keys = uniform_keys(seed, n_keys, g0, n)
    p = permits(seed, g0, n, p_lo, p_hi)
    ts = batch_timestamps(batch, n, interval_us, t0_us)
    return keys, p, ts
