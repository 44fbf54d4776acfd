"""Python host mirror of the engine (tests, bench).  Every decision runs in the HIP
engine through the C ABI (``_capi``); this module only moves buffers.

``TokenBucketEngine`` corresponds to one ``RedisTokenBucketRateLimiterOptions`` /
``PartitionedRedisTokenBucketRateLimiter`` instance of the reference
(TokenBucket/PartitionedRedisTokenBucketRateLimiter.cs:7-55), with the per-request
``ScriptEvaluateAsync`` (PTB:42) replaced by ``acquire_batch``.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_double, c_int32, c_uint32, c_void_p
from typing import Optional, Tuple

import numpy as np

from . import _capi
from ._capi import TbeError


def fill_rate(tokens_per_period: int, period_ticks: int) -> float:
    return _capi.load().tbe_fill_rate(tokens_per_period, period_ticks)


class TokenBucketEngine:
    def __init__(self, n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                 device: int = -1, stage_timing: bool = False, max_batch: int = 0):
        self._lib = _capi.load()
        flags = _capi.TBE_FLAG_STAGE_TIMING if stage_timing else 0
        self.config = _capi.make_config(n_keys, token_limit, tokens_per_period, period_ticks,
                                        device=device, flags=flags, max_batch=max_batch)
        h = c_void_p()
        st = self._lib.tbe_create(byref(self.config), byref(h))
        if st != _capi.TBE_OK:
            raise TbeError(st, "tbe_create failed")
        self._h = h
        self.n_keys = n_keys

    # ------------------------------------------------------------------ lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tbe_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int) -> None:
        if st != _capi.TBE_OK:
            msg = self._lib.tbe_last_error(self._h).decode() if self._h else "disposed"
            raise TbeError(st, msg)

    @property
    def handle(self) -> c_void_p:
        if not self._h:
            raise TbeError(_capi.TBE_EDISPOSED, "engine disposed")
        return self._h

    # ------------------------------------------------------------------ decisions
    def acquire_batch(self, keys, permits, ts_us) -> Tuple[np.ndarray, np.ndarray]:
        """Host arrays in, host arrays out (granted u8, remaining i32), arrival order."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        if permits.shape[0] != n or ts_us.shape[0] != n:
            raise ValueError("keys, permits and ts_us must have the same length")
        granted = np.empty(n, dtype=np.uint8)
        remaining = np.empty(n, dtype=np.int32)
        self._check(self._lib.tbe_acquire_batch(
            self.handle, keys.ctypes.data, permits.ctypes.data, ts_us.ctypes.data, n,
            granted.ctypes.data, remaining.ctypes.data))
        return granted, remaining

    def acquire_batch_device(self, d_keys, d_permits, d_ts, d_granted, d_remaining,
                             stream: Optional[int] = None) -> None:
        """Device tensors (torch, on this engine's GPU); enqueued, not synchronised."""
        n = d_keys.numel()
        self._check(self._lib.tbe_acquire_batch_device(
            self.handle, d_keys.data_ptr(), d_permits.data_ptr(), d_ts.data_ptr(), n,
            d_granted.data_ptr(), d_remaining.data_ptr(), stream))

    def synchronize(self) -> None:
        self._check(self._lib.tbe_synchronize(self.handle))

    # ------------------------------------------------------------------ state
    def query(self, key: int, ts_us: int = -1) -> Optional[Tuple[float, float]]:
        v, t, present = c_double(), c_double(), c_int32()
        self._check(self._lib.tbe_query(self.handle, key, ts_us, byref(v), byref(t), byref(present)))
        return (v.value, t.value) if present.value else None

    def export_state(self, first: int = 0, count: Optional[int] = None):
        if count is None:
            count = self.n_keys - first
        v = np.empty(count, dtype=np.float64)
        t = np.empty(count, dtype=np.int64)
        self._check(self._lib.tbe_export_state(self.handle, first, count, v.ctypes.data,
                                               t.ctypes.data))
        return v, t

    def stage_times(self) -> dict:
        out = (c_double * len(_capi.STAGES))()
        nw = c_uint32()
        self._check(self._lib.tbe_stage_times(self.handle, out, len(_capi.STAGES), byref(nw)))
        return {name: out[i] for i, name in enumerate(_capi.STAGES[: nw.value])}
