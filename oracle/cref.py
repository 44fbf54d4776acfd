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
