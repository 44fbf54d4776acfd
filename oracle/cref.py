"""ctypes wrapper of the C restatement (oracle/tb_ref.c).  TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_uint64, c_void_p

import numpy as np

from .build import LIB, build_oracle

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build_oracle()
    lib = ctypes.CDLL(LIB)
    lib.tbr_new_t.restype = c_double
    lib.tbr_new_t.argtypes = [c_int64]
    lib.tbr_fill_rate.restype = c_double
    lib.tbr_fill_rate.argtypes = [c_int32, c_int64]
    lib.tbr_ttl_seconds.restype = c_int64
    lib.tbr_ttl_seconds.argtypes = [c_int32, c_double]
    lib.tbr_create.restype = c_void_p
    lib.tbr_create.argtypes = [c_uint64, c_int32, c_double]
    lib.tbr_destroy.restype = None
    lib.tbr_destroy.argtypes = [c_void_p]
    lib.tbr_acquire_batch.restype = c_int
    lib.tbr_acquire_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                      c_void_p]
    lib.tbr_acquire_batch_mt.restype = c_int
    lib.tbr_acquire_batch_mt.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                         c_void_p, c_int]
    lib.tbr_query.restype = c_int
    lib.tbr_query.argtypes = [c_void_p, c_uint64, c_int64, POINTER(c_double), POINTER(c_double)]
    lib.tbr_export.restype = None
    lib.tbr_export.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.tbr_gen_uniform_keys.restype = None
    lib.tbr_gen_uniform_keys.argtypes = [c_uint64, c_uint64, c_uint64, c_uint64, c_void_p]
    lib.tbr_gen_permits.restype = None
    lib.tbr_gen_permits.argtypes = [c_uint64, c_uint64, c_uint64, c_int32, c_int32, c_void_p]
    lib.tbr_gen_timestamps.restype = None
    lib.tbr_gen_timestamps.argtypes = [c_int64, c_uint64, c_int64, c_int64, c_void_p]
    _lib = lib
    return lib


class CTokenBucket:
    """C restatement of the TB acquire script over a dense key table."""

    def __init__(self, n_keys: int, token_limit: int, fill_rate: float):
        self._lib = load()
        self._h = self._lib.tbr_create(n_keys, token_limit, fill_rate)
        if not self._h:
            raise ValueError("tbr_create rejected the configuration")
        self.n_keys = n_keys

    def close(self):
        if self._h:
            self._lib.tbr_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def acquire_batch(self, keys, permits, ts_us, threads: int = 1):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        granted = np.empty(n, dtype=np.uint8)
        remaining = np.empty(n, dtype=np.int32)
        rc = self._lib.tbr_acquire_batch_mt(self._h, keys.ctypes.data, permits.ctypes.data,
                                            ts_us.ctypes.data, n, granted.ctypes.data,
                                            remaining.ctypes.data, threads)
        if rc != 0:
            raise ValueError("invalid request in batch")
        return granted, remaining

    def query(self, key: int, ts_us: int = -1):
        v, t = c_double(), c_double()
        ok = self._lib.tbr_query(self._h, key, ts_us, ctypes.byref(v), ctypes.byref(t))
        return (v.value, t.value) if ok else None

    def export_state(self):
        v = np.empty(self.n_keys, dtype=np.float64)
        t = np.empty(self.n_keys, dtype=np.int64)
        self._lib.tbr_export(self._h, v.ctypes.data, t.ctypes.data)
        return v, t


def gen_batch(seed: int, n_keys: int, batch: int, n: int, interval_us: int, p_lo: int = 1,
              p_hi: int = 1, t0_us: int = 1_760_000_000_000_000):
    lib = load()
    keys = np.empty(n, dtype=np.uint64)
    permits = np.empty(n, dtype=np.int32)
    ts = np.empty(n, dtype=np.int64)
    g0 = batch * n
    lib.tbr_gen_uniform_keys(seed, n_keys, g0, n, keys.ctypes.data)
    lib.tbr_gen_permits(seed, g0, n, p_lo, p_hi, permits.ctypes.data)
    lib.tbr_gen_timestamps(batch, n, interval_us, t0_us, ts.ctypes.data)
    return keys, permits, ts


class CQueueingTokenBucket:
    """C restatement of the TokenBucketWithQueue spec (oracle/tb_ref.c tbrq_*)."""

    def __init__(self, n_keys: int, token_limit: int, fill_rate: float, queue_limit: int, order: int):
        lib = load()
        lib.tbrq_create.restype = c_void_p
        lib.tbrq_create.argtypes = [c_uint64, c_int32, c_double, c_int32, c_int32]
        lib.tbrq_destroy.argtypes = [c_void_p]
        lib.tbrq_acquire_batch.restype = c_int
        lib.tbrq_acquire_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int64,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]
        lib.tbrq_refresh.restype = c_int
        lib.tbrq_refresh.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]
        lib.tbrq_queue_of.restype = ctypes.c_uint32
        lib.tbrq_queue_of.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, ctypes.c_uint32]
        lib.tbrq_bucket_table.restype = c_void_p
        lib.tbrq_bucket_table.argtypes = [c_void_p]
        lib.tbrq_acquire_batch_mt.restype = c_int
        lib.tbrq_acquire_batch_mt.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int64,
                                              c_void_p, c_void_p, c_int, c_void_p]
        lib.tbrq_refresh_mt.restype = c_int
        lib.tbrq_refresh_mt.argtypes = [c_void_p, c_int64, c_int, c_void_p]
        lib.tbrq_mt_log.restype = c_uint64
        lib.tbrq_mt_log.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64]
        self._lib = lib
        self._h = lib.tbrq_create(n_keys, token_limit, fill_rate, queue_limit, order)
        if not self._h:
            raise ValueError("tbrq_create rejected the configuration")
        self.n_keys, self.queue_limit = n_keys, queue_limit

    def close(self):
        if self._h:
            self._lib.tbrq_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _mt_log(self, m: int):
        a = np.empty(m, np.uint64)
        ids = np.empty(m, np.int64)
        rem = np.empty(m, np.int32)
        got = self._lib.tbrq_mt_log(a.ctypes.data, ids.ctypes.data, rem.ctypes.data, m)
        assert got == m
        return a, ids, rem

    def acquire_batch(self, keys, permits, ts_us, id_base: int, threads: int = 1):
        """(status, remaining, eviction causes, evicted ids); threads > 1: key-sharded
        (tbrq_acquire_batch_mt), evictions then sorted by (cause, id)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        status = np.empty(n, np.uint8)
        remaining = np.empty(n, np.int32)
        if threads > 1:
            n_ev = ctypes.c_uint64()
            rc = self._lib.tbrq_acquire_batch_mt(self._h, keys.ctypes.data, permits.ctypes.data,
                                                 ts_us.ctypes.data, n, id_base, status.ctypes.data,
                                                 remaining.ctypes.data, threads, ctypes.byref(n_ev))
            if rc != 0:
                raise ValueError(f"tbrq_acquire_batch_mt failed ({rc})")
            cause, ids, _ = self._mt_log(n_ev.value)
            o = np.lexsort((ids, cause))
            return status, remaining, cause[o], ids[o]
        max_ev = n * max(1, self.queue_limit) + 1
        ev_id = np.empty(max_ev, np.int64)
        ev_cause = np.empty(max_ev, np.uint64)
        n_ev = ctypes.c_uint64()
        rc = self._lib.tbrq_acquire_batch(self._h, keys.ctypes.data, permits.ctypes.data,
                                          ts_us.ctypes.data, n, id_base, status.ctypes.data,
                                          remaining.ctypes.data, ev_id.ctypes.data,
                                          ev_cause.ctypes.data, max_ev, ctypes.byref(n_ev))
        if rc != 0:
            raise ValueError("invalid request in batch")
        m = n_ev.value
        return status, remaining, ev_cause[:m].copy(), ev_id[:m].copy()

    def refresh(self, ts_us: int, threads: int = 1):
        if threads > 1:
            nl = ctypes.c_uint64()
            rc = self._lib.tbrq_refresh_mt(self._h, ts_us, threads, ctypes.byref(nl))
            if rc != 0:
                raise ValueError(f"tbrq_refresh_mt failed ({rc})")
            return self._mt_log(nl.value)
        cap = int(self.n_keys) * max(1, self.queue_limit)
        cap = min(cap, 1 << 26)
        lk = np.empty(cap, np.uint64)
        lid = np.empty(cap, np.int64)
        lrem = np.empty(cap, np.int32)
        nl = ctypes.c_uint64()
        rc = self._lib.tbrq_refresh(self._h, ts_us, lk.ctypes.data, lid.ctypes.data, lrem.ctypes.data,
                                    cap, ctypes.byref(nl))
        if rc != 0:
            raise ValueError("invalid refresh")
        m = min(nl.value, cap)
        return lk[:m].copy(), lid[:m].copy(), lrem[:m].copy()

    def cancel(self, keys, ids) -> np.ndarray:
        """tbrq_cancel per (key, request id) pair in order: 1 where it was queued."""
        self._lib.tbrq_cancel.restype = c_int
        self._lib.tbrq_cancel.argtypes = [c_void_p, c_uint64, c_int64]
        return np.array([self._lib.tbrq_cancel(self._h, int(k), int(i))
                         for k, i in zip(np.asarray(keys).tolist(), np.asarray(ids).tolist())], dtype=np.uint8)

    def queue_of(self, key: int):
        ids = np.empty(max(1, self.queue_limit), np.int64)
        ps = np.empty(max(1, self.queue_limit), np.int32)
        c = self._lib.tbrq_queue_of(self._h, key, ids.ctypes.data, ps.ctypes.data, ids.size)
        return list(zip(ids[:c].tolist(), ps[:c].tolist()))

    def bucket_state(self):
        v = np.empty(self.n_keys, dtype=np.float64)
        t = np.empty(self.n_keys, dtype=np.int64)
        self._lib.tbr_export(self._lib.tbrq_bucket_table(self._h), v.ctypes.data, t.ctypes.data)
        return v, t


class CApprox:
    """C restatement of one ApproximateTokenBucket client for every key plus its replica of
    the global tier (oracle/tb_ref.c tba_*): the config-E checker and CPU baseline."""

    def __init__(self, n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                 queue_limit: int = 0, order: int = 0, zero_slots: int = 4):
        lib = load()
        lib.tba_create.restype = c_void_p
        lib.tba_create.argtypes = [c_uint64, c_int32, c_int32, c_int64, c_int32, c_int32, c_int32]
        lib.tba_destroy.argtypes = [c_void_p]
        lib.tba_acquire_batch.restype = c_int
        lib.tba_acquire_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_int, c_int64, c_void_p,
                                          c_void_p, c_int, c_void_p]
        lib.tba_collect.argtypes = [c_void_p, c_void_p]
        lib.tba_sync.restype = c_int
        lib.tba_sync.argtypes = [c_void_p, c_void_p, ctypes.c_uint32, ctypes.c_uint32, c_int64, c_int64, c_int,
                                 c_void_p]
        lib.tba_export.argtypes = [c_void_p] + [c_void_p] * 8
        lib.tba_queue_of.restype = ctypes.c_uint32
        lib.tba_queue_of.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, ctypes.c_uint32]
        lib.tbrq_mt_log.restype = c_uint64
        lib.tbrq_mt_log.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64]
        self._lib = lib
        self._h = lib.tba_create(n_keys, token_limit, tokens_per_period, period_ticks, queue_limit, order,
                                 zero_slots)
        if not self._h:
            raise ValueError("tba_create rejected the configuration")
        self.n_keys, self.queue_limit, self.zero_slots = n_keys, queue_limit, zero_slots

    def close(self):
        if self._h:
            self._lib.tba_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _log(self, m: int):
        a = np.empty(m, np.uint64)
        ids = np.empty(m, np.int64)
        rem = np.empty(m, np.int32)
        assert self._lib.tbrq_mt_log(a.ctypes.data, ids.ctypes.data, rem.ctypes.data, m) == m
        return a, ids, rem

    def acquire_batch(self, keys, permits, wait: bool = True, id_base: int = 0, threads: int = 1):
        """(status u8, available i32, eviction causes u64, evicted ids i64), evictions
        sorted by (cause, id) as the engine reports them."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        n = keys.shape[0]
        status = np.empty(n, np.uint8)
        avail = np.empty(n, np.int32)
        n_ev = ctypes.c_uint64()
        rc = self._lib.tba_acquire_batch(self._h, keys.ctypes.data, permits.ctypes.data, n, 1 if wait else 0,
                                         id_base, status.ctypes.data, avail.ctypes.data, threads,
                                         ctypes.byref(n_ev))
        if rc != 0:
            raise ValueError(f"tba_acquire_batch failed ({rc})")
        cause, ids, _ = self._log(n_ev.value)
        o = np.lexsort((ids, cause))
        return status, avail, cause[o], ids[o]

    def collect(self) -> np.ndarray:
        out = np.empty(self.n_keys, np.int32)
        self._lib.tba_collect(self._h, out.ctypes.data)
        return out

    def sync(self, all_counts, n_clients: int, my: int, ts_us: int, stagger_us: int, threads: int = 1):
        """Drain log (keys u64, request ids i64, available i32) in key order."""
        c = np.ascontiguousarray(all_counts, dtype=np.int32)
        assert c.size == n_clients * self.n_keys
        nl = ctypes.c_uint64()
        rc = self._lib.tba_sync(self._h, c.ctypes.data, n_clients, my, ts_us, stagger_us, threads,
                                ctypes.byref(nl))
        if rc != 0:
            raise ValueError(f"tba_sync failed ({rc})")
        return self._log(nl.value)

    def export(self):
        """dict of per-key arrays: local, global, est, available, queued, v, p, t_us."""
        n = self.n_keys
        out = {"local": np.empty(n, np.int32), "global": np.empty(n, np.int32), "est": np.empty(n, np.float64),
               "available": np.empty(n, np.int32), "queued": np.empty(n, np.uint32),
               "v": np.empty(n, np.float64), "p": np.empty(n, np.float64), "t_us": np.empty(n, np.int64)}
        self._lib.tba_export(self._h, *[out[k].ctypes.data for k in
                                        ("local", "global", "est", "available", "queued", "v", "p", "t_us")])
        return out

    def cancel(self, keys, ids) -> np.ndarray:
        """tba_cancel per (key, request id) pair in order: 1 where it was queued."""
        self._lib.tba_cancel.restype = c_int
        self._lib.tba_cancel.argtypes = [c_void_p, c_uint64, c_int64]
        return np.array([self._lib.tba_cancel(self._h, int(k), int(i))
                         for k, i in zip(np.asarray(keys).tolist(), np.asarray(ids).tolist())], dtype=np.uint8)

    def queue_of(self, key: int):
        cap = max(1, self.queue_limit) + self.zero_slots
        ids = np.empty(cap, np.int64)
        ps = np.empty(cap, np.int32)
        c = self._lib.tba_queue_of(self._h, key, ids.ctypes.data, ps.ctypes.data, cap)
        return list(zip(ids[:c].tolist(), ps[:c].tolist()))
