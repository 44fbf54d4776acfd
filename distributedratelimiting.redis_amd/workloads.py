"""Synthetic request workloads for bench.py and the tests.

Generation only: nothing here decides a request.  Config B's uniform stream is
generated on the device (``tbe_gen_batch_device``); config C's skewed key stream is
drawn here on the host and copied to HBM before any timed region.

Config C: keys follow a bounded Zipf(s = 1.1) law over the key space (rank 1 is the
hottest key), and ranks map to key ids through a fixed bijection, so the hot keys land
in unrelated partition buckets.  The reference ships no workload generator (it has no
tests or benchmarks); this one is the build's own.
"""
from __future__ import annotations

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1
STREAM_ZIPF = 0x3C3C3C3C3C3C3C3C


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(M1)
        z ^= z >> np.uint64(27)
        z *= np.uint64(M2)
        z ^= z >> np.uint64(31)
    return z


def _uniform01(seed: int, stream_id: int, g: np.ndarray) -> np.ndarray:
    """U[0, 1) doubles from the splitmix64 counter stream (53 random bits)."""
    base = np.uint64((seed ^ stream_id) & MASK64)
    with np.errstate(over="ignore"):
        r = _mix64(base + g.astype(np.uint64) * np.uint64(GAMMA))
    return (r >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def _helper1(x):
    ax = np.abs(x)
    safe = np.where(ax > 1e-8, x, 1.0)
    return np.where(ax > 1e-8, np.log1p(safe) / safe, 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x)))


def _helper2(x):
    ax = np.abs(x)
    safe = np.where(ax > 1e-8, x, 1.0)
    return np.where(ax > 1e-8, np.expm1(safe) / safe,
                    1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x)))


class ZipfSampler:
    """Zipf(s) on {1..n_items} by rejection-inversion (Hörmann & Derflinger, 1996),
    vectorised.  Deterministic: draw g of a stream uses counter g (and a fresh stream
    per rejection round), so a batch is a pure function of (seed, g0, n)."""

    def __init__(self, n_items: int, s: float = 1.1):
        if n_items < 1 or s <= 0.0:
            raise ValueError("need n_items >= 1 and s > 0")
        self.n, self.s = int(n_items), float(s)
        self.h_x1 = self._hint(np.float64(1.5)) - 1.0
        self.h_n = self._hint(np.float64(self.n + 0.5))
        self.sq = 2.0 - self._hinv(self._hint(np.float64(2.5)) - self._h(np.float64(2.0)))

    def _h(self, x):
        return np.exp(-self.s * np.log(x))

    def _hint(self, x):
        lx = np.log(x)
        return _helper2((1.0 - self.s) * lx) * lx

    def _hinv(self, x):
        t = np.maximum(x * (1.0 - self.s), -1.0)
        return np.exp(_helper1(t) * x)

    def ranks(self, seed: int, g0: int, n: int) -> np.ndarray:
        out = np.empty(n, dtype=np.int64)
        todo = np.arange(n, dtype=np.int64)
        attempt = 0
        while todo.size:
            u01 = _uniform01(seed, (STREAM_ZIPF + attempt) & MASK64, g0 + todo)
            u = self.h_n + u01 * (self.h_x1 - self.h_n)
            x = self._hinv(u)
            k = np.clip(np.floor(x + 0.5), 1, self.n)
            ok = (k - x <= self.sq) | (u >= self._hint(k + 0.5) - self._h(k))
            out[todo[ok]] = k[ok].astype(np.int64)
            todo = todo[~ok]
            attempt += 1
        return out


def _scramble(x: np.ndarray, bits: int) -> np.ndarray:
    """A fixed bijection of [0, 2^bits): odd multiply-add then xorshift, three rounds."""
    mask = np.uint64((1 << bits) - 1)
    sh = np.uint64(max(1, bits // 2))
    with np.errstate(over="ignore"):
        for a, c in ((0x9E3779B97F4A7C15, 0x632BE59BD9B4E019),
                     (0xD1B54A32D192ED03, 0x8CB92BA72F3D8DD7),
                     (0xAEF17502108EF2D9, 0x2545F4914F6CDD1D)):
            x = (x * np.uint64(a) + np.uint64(c)) & mask
            x ^= x >> sh
    return x


def rank_to_key(ranks: np.ndarray, n_keys: int) -> np.ndarray:
    """Bijection rank (1..n_keys) -> key id in [0, n_keys) by cycle walking."""
    bits = max(1, int(n_keys - 1).bit_length())
    x = _scramble((ranks - 1).astype(np.uint64), bits)
    bad = x >= np.uint64(n_keys)
    while bad.any():
        x[bad] = _scramble(x[bad], bits)
        bad = x >= np.uint64(n_keys)
    return x


def zipf_keys(seed: int, n_keys: int, g0: int, n: int, s: float = 1.1,
              sampler: ZipfSampler | None = None) -> np.ndarray:
    """n keys (u64) of a Zipf(s) request stream over [0, n_keys), draws g0 .. g0+n-1."""
    sampler = sampler or ZipfSampler(n_keys, s)
    return rank_to_key(sampler.ranks(seed, g0, n), n_keys)


def batch_timestamps(batch: int, n: int, interval_us: int, t0_us: int) -> np.ndarray:
    """batch b spans interval_us from t0 + b*interval, non-decreasing."""
    i = np.arange(n, dtype=np.int64)
    return t0_us + batch * interval_us + (i * interval_us) // n
