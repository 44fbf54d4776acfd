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


class PinnedArray:
    """A numpy array over page-locked host memory from ``tbe_alloc_host`` (the host-buffer
    calls copy it by DMA).  ``.array`` is valid until ``free()`` or collection of this
    object; keep the object alive while the array (or a view of it) is in use."""

    def __init__(self, n: int, dtype):
        self._lib = _capi.load()
        dt = np.dtype(dtype)
        nbytes = max(1, int(n) * dt.itemsize)
        p = c_void_p()
        st = self._lib.tbe_alloc_host(nbytes, byref(p))
        if st != 0 or not p.value:
            raise TbeError(st, f"tbe_alloc_host({nbytes}) failed")
        self._ptr = p.value
        buf = (ctypes.c_uint8 * nbytes).from_address(self._ptr)
        self.array = np.frombuffer(buf, dtype=np.uint8)[: int(n) * dt.itemsize].view(dt)

    def free(self) -> None:
        if self._ptr:
            self.array = None
            self._lib.tbe_free_host(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class TokenBucketEngine:
    KIND = _capi.TBE_KIND_TOKEN_BUCKET

    def __init__(self, n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                 device: int = -1, stage_timing: bool = False, max_batch: int = 0,
                 queue_limit: int = 0, queue_order: int = 0, pack: bool = True, hot: bool = True,
                 pipeline: bool = True, narrow: bool = True, zero_wait_slots: int = 0,
                 fold_records: bool = True, digit_stream: bool = True, rerank: bool = False):
        self._lib = _capi.load()
        # stage_timing: True (every stage), "fold" (the fold alone) or False
        flags = (_capi.TBE_FLAG_FOLD_TIMING if stage_timing == "fold"
                 else _capi.TBE_FLAG_STAGE_TIMING if stage_timing else 0)
        if not pack:
            flags |= _capi.TBE_FLAG_NO_PACK
        if not hot:
            flags |= _capi.TBE_FLAG_NO_HOT
        if not pipeline:
            flags |= _capi.TBE_FLAG_NO_PIPELINE
        if not narrow:
            flags |= _capi.TBE_FLAG_NO_NARROW
        if not fold_records:
            flags |= _capi.TBE_FLAG_UNSCATTER_ALL
        if not digit_stream:
            flags |= _capi.TBE_FLAG_HIST_RECORDS
        if rerank:
            flags |= _capi.TBE_FLAG_RERANK
        self.config = _capi.make_config(n_keys, token_limit, tokens_per_period, period_ticks,
                                        kind=self.KIND, queue_limit=queue_limit,
                                        queue_order=queue_order, device=device, flags=flags,
                                        max_batch=max_batch, zero_wait_slots=zero_wait_slots)
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
    def acquire_batch(self, keys, permits, ts_us, granted=None, remaining=None) -> Tuple[np.ndarray, np.ndarray]:
        """Host arrays in, host arrays out (granted u8, remaining i32), arrival order.
        granted/remaining: optional output arrays (e.g. PinnedArray.array: with every
        buffer page-locked, large batches take the chunked path whose copies overlap the
        decisions)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        if permits.shape[0] != n or ts_us.shape[0] != n:
            raise ValueError("keys, permits and ts_us must have the same length")
        granted = np.empty(n, dtype=np.uint8) if granted is None else granted
        remaining = np.empty(n, dtype=np.int32) if remaining is None else remaining
        if granted.shape != (n,) or remaining.shape != (n,) or granted.dtype != np.uint8 or \
                remaining.dtype != np.int32 or not (granted.flags.c_contiguous and remaining.flags.c_contiguous):
            raise ValueError("granted must be u8[n] and remaining i32[n], contiguous")
        self._check(self._lib.tbe_acquire_batch(
            self.handle, keys.ctypes.data, permits.ctypes.data, ts_us.ctypes.data, n,
            granted.ctypes.data, remaining.ctypes.data))
        return granted, remaining

    def acquire_batch_device(self, d_keys, d_permits, d_ts, d_granted, d_remaining,
                             stream: Optional[int] = None) -> None:
        """Device tensors (torch, on this engine's GPU); enqueued, not synchronised.
        stream=None: the inputs must be complete now and the replies are complete at
        ``synchronize()``; a stream handle orders both on that stream (tbe.h)."""
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

    def import_state(self, v, t_us, first: int = 0) -> None:
        """Restore rows [first, first + len) from an export_state snapshot (tbe_import_state)."""
        v = np.ascontiguousarray(v, dtype=np.float64)
        t_us = np.ascontiguousarray(t_us, dtype=np.int64)
        if v.shape != t_us.shape:
            raise ValueError("v and t_us must have the same length")
        self._check(self._lib.tbe_import_state(self.handle, first, v.shape[0], v.ctypes.data,
                                               t_us.ctypes.data))

    def layout(self) -> dict:
        """{passes, r_bits, packed, hot, pipeline, narrow, medium, fold_records, digit_stream, rerank,
        narrow_pass0, queue_header_32} of this engine's
        batch pipeline (tbe_layout)."""
        a, b, c = c_uint32(), c_uint32(), c_uint32()
        self._check(self._lib.tbe_layout(self.handle, byref(a), byref(b), byref(c)))
        return {"passes": a.value, "r_bits": b.value, "packed": bool(c.value & 1),
                "hot": bool(c.value & 2), "pipeline": bool(c.value & 4), "narrow": bool(c.value & 8),
                "medium": bool(c.value & 16), "fold_records": bool(c.value & 32),
                "digit_stream": bool(c.value & 64), "rerank": bool(c.value & 128),
                "narrow_pass0": bool(c.value & 256), "queue_header_32": bool(c.value & 512)}

    def batch_format(self, n: int) -> dict:
        """The record layout a batch of n requests takes (tbe_batch_format)."""
        out = (c_uint32 * 9)()
        self._check(self._lib.tbe_batch_format(self.handle, n, out, 9))
        names = ("passes", "fold_records", "position_bits", "fold_time_bits", "key_bits", "permit_bits",
                 "pass0_time_bits", "r_bits", "sparse")
        return {k: (bool(out[i]) if k in ("fold_records", "sparse") else out[i]) for i, k in enumerate(names)}

    def stage_times(self) -> dict:
        out = (c_double * len(_capi.STAGES))()
        nw = c_uint32()
        self._check(self._lib.tbe_stage_times(self.handle, out, len(_capi.STAGES), byref(nw)))
        return {name: out[i] for i, name in enumerate(_capi.STAGES[: nw.value])}


class QueueingTokenBucketEngine(TokenBucketEngine):
    """TokenBucketWithQueue (TokenBucketWithQueue/RedisTokenBucketRateLimiter.cs, Q):
    WaitAsyncCore (Q:67-134) as ``wait_batch``, the timer drain (Q:237-271) as ``refresh``."""

    KIND = _capi.TBE_KIND_QUEUEING

    def __init__(self, n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                 queue_limit: int, queue_order: int = 0, **kw):
        super().__init__(n_keys, token_limit, tokens_per_period, period_ticks,
                         queue_limit=queue_limit, queue_order=queue_order, **kw)
        self.queue_limit = queue_limit

    def wait_batch(self, keys, permits, ts_us, id_base: int, status=None, remaining=None):
        """Returns (status u8, remaining i32, evicted (cause index u64, request id i64)).
        `status` / `remaining` may be caller arrays (e.g. PinnedArray: with page-locked
        inputs too, batches of >= 2 chunks take the overlapped chunked path)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        status = np.empty(n, dtype=np.uint8) if status is None else status
        remaining = np.empty(n, dtype=np.int32) if remaining is None else remaining
        n_ev = ctypes.c_uint64()
        self._check(self._lib.tbe_wait_batch(self.handle, keys.ctypes.data, permits.ctypes.data,
                                             ts_us.ctypes.data, n, id_base, status.ctypes.data,
                                             remaining.ctypes.data, byref(n_ev)))
        m = n_ev.value
        cause = np.empty(m, dtype=np.uint64)
        ids = np.empty(m, dtype=np.int64)
        nw = ctypes.c_uint64()
        if m:
            self._check(self._lib.tbe_evicted(self.handle, cause.ctypes.data, ids.ctypes.data, m, byref(nw)))
        return status, remaining, (cause, ids)

    def attempt_batch(self, keys, permits, ts_us):
        """AttemptAcquire (lease or fail, never queue); returns (status u8, remaining i32)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        ts_us = np.ascontiguousarray(ts_us, dtype=np.int64)
        n = keys.shape[0]
        status = np.empty(n, dtype=np.uint8)
        remaining = np.empty(n, dtype=np.int32)
        self._check(self._lib.tbe_queue_attempt_batch(self.handle, keys.ctypes.data, permits.ctypes.data,
                                                      ts_us.ctypes.data, n, status.ctypes.data,
                                                      remaining.ctypes.data))
        return status, remaining

    def wait_batch_device(self, d_keys, d_permits, d_ts, d_status, d_remaining, id_base: int,
                          wait: bool = True, stream: Optional[int] = None) -> None:
        """Device tensors in and out; enqueued, not synchronised (tbe_wait_batch_device).
        NewestFirst evictions: ``evicted()`` after the call."""
        n = d_keys.numel()
        self._check(self._lib.tbe_wait_batch_device(
            self.handle, d_keys.data_ptr(), d_permits.data_ptr(), d_ts.data_ptr(), n, id_base,
            1 if wait else 0, d_status.data_ptr(), d_remaining.data_ptr(), stream))

    def evicted(self):
        """(cause index u64, request id i64) of the last wait batch, sorted (tbe_evicted)."""
        nw = ctypes.c_uint64()
        self._check(self._lib.tbe_evicted(self.handle, None, None, 0, byref(nw)))
        # capacity 0 fetched the log; a second call copies it out
        cap = 1 << 20
        while True:
            cause = np.empty(cap, dtype=np.uint64)
            ids = np.empty(cap, dtype=np.int64)
            self._check(self._lib.tbe_evicted(self.handle, cause.ctypes.data, ids.ctypes.data, cap,
                                              byref(nw)))
            if nw.value < cap:
                return cause[: nw.value], ids[: nw.value]
            cap *= 4

    def refresh_bound(self) -> int:
        b = ctypes.c_uint64()
        self._check(self._lib.tbe_refresh_bound(self.handle, byref(b)))
        return b.value

    def refresh_device(self, ts_us: int, d_keyseq, d_ids, d_rem, d_count,
                       stream: Optional[int] = None) -> None:
        """Enqueue one replenish tick; the drain log lands in the device tensors
        (capacity = d_keyseq.numel(), which must be >= refresh_bound())."""
        self._check(self._lib.tbe_refresh_device(self.handle, ts_us, d_keyseq.data_ptr(), d_ids.data_ptr(),
                                                 d_rem.data_ptr(), d_keyseq.numel(), d_count.data_ptr(),
                                                 stream))

    def wait_batch_tick_device(self, d_keys, d_permits, d_ts, d_status, d_remaining, id_base: int,
                               tick_ts_us: int, d_keyseq, d_ids, d_rem, d_count, wait: bool = True,
                               stream: Optional[int] = None) -> None:
        """``wait_batch_device`` then ``refresh_device(tick_ts_us)`` as one fused call
        (tbe_wait_batch_tick_device); the log capacity must cover ``refresh_bound()`` after
        the batch."""
        n = d_keys.numel()
        self._check(self._lib.tbe_wait_batch_tick_device(
            self.handle, d_keys.data_ptr(), d_permits.data_ptr(), d_ts.data_ptr(), n, id_base,
            1 if wait else 0, d_status.data_ptr(), d_remaining.data_ptr(), tick_ts_us, d_keyseq.data_ptr(),
            d_ids.data_ptr(), d_rem.data_ptr(), d_keyseq.numel(), d_count.data_ptr(), stream))

    def refresh(self, ts_us: int):
        """One replenish tick; returns (keys u64, request ids i64, remaining i32) in (key, drain) order."""
        n = ctypes.c_uint64()
        self._check(self._lib.tbe_refresh(self.handle, ts_us, byref(n)))
        m = n.value
        keys = np.empty(m, dtype=np.uint64)
        ids = np.empty(m, dtype=np.int64)
        rem = np.empty(m, dtype=np.int32)
        nw = ctypes.c_uint64()
        if m:
            self._check(self._lib.tbe_refresh_log(self.handle, keys.ctypes.data, ids.ctypes.data,
                                                  rem.ctypes.data, m, byref(nw)))
        return keys, ids, rem

    def queue_of(self, key: int):
        cap = max(1, self.queue_limit) + getattr(self, "zero_wait_slots", 0)
        ids = np.empty(cap, dtype=np.int64)
        ps = np.empty(cap, dtype=np.int32)
        cnt = c_uint32()
        self._check(self._lib.tbe_queue_of(self.handle, key, ids.ctypes.data, ps.ctypes.data, cap,
                                           byref(cnt)))
        c = min(cnt.value, cap)
        return list(zip(ids[:c].tolist(), ps[:c].tolist()))

    def cancel(self, keys, request_ids):
        """Cancel queued requests (CancelQueueState.TrySetCanceled, Q:480-506 / A:531-557;
        tbe_queue_cancel); returns u8[n], 1 where the request was queued and is removed."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        request_ids = np.ascontiguousarray(request_ids, dtype=np.int64)
        n = keys.shape[0]
        if request_ids.shape[0] != n:
            raise ValueError("keys and request_ids differ in length")
        out = np.empty(n, dtype=np.uint8)
        m = ctypes.c_uint64()
        self._check(self._lib.tbe_queue_cancel(self.handle, keys.ctypes.data, request_ids.ctypes.data,
                                               n, out.ctypes.data, byref(m)))
        return out


class ApproximateEngine(QueueingTokenBucketEngine):
    """ApproximateTokenBucket (ApproximateTokenBucket/RedisApproximateTokenBucketRateLimiter.cs, A):
    one client's local tier for every key plus a replica of the shared global tier.
    ``acquire_batch`` = AcquireCore / WaitAsyncCore (A:84-183); a refresh epoch =
    ``collect`` (A:430-435) -> exchange the counts between clients (RCCL all-gather, or
    all-reduce for one node-wide client) -> ``sync`` (A:439-508)."""

    KIND = _capi.TBE_KIND_APPROXIMATE

    def __init__(self, n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                 queue_limit: int, queue_order: int = 0, zero_wait_slots: int = 4, **kw):
        """zero_wait_slots: queue entries per key for zero-permit waits (tbe.h)."""
        super().__init__(n_keys, token_limit, tokens_per_period, period_ticks, queue_limit,
                         queue_order, zero_wait_slots=zero_wait_slots, **kw)
        self.zero_wait_slots = zero_wait_slots

    def acquire_batch(self, keys, permits, wait: bool = True, id_base: int = 0, status=None, available=None):
        """Returns (status u8, available i32, evicted (cause index, request id))."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        permits = np.ascontiguousarray(permits, dtype=np.int32)
        n = keys.shape[0]
        status = np.empty(n, dtype=np.uint8) if status is None else status
        avail = np.empty(n, dtype=np.int32) if available is None else available
        n_ev = ctypes.c_uint64()
        self._check(self._lib.tbe_approx_acquire_batch(self.handle, keys.ctypes.data, permits.ctypes.data,
                                                       n, 1 if wait else 0, id_base, status.ctypes.data,
                                                       avail.ctypes.data, byref(n_ev)))
        m = n_ev.value
        cause = np.empty(m, dtype=np.uint64)
        ids = np.empty(m, dtype=np.int64)
        nw = ctypes.c_uint64()
        if m:
            self._check(self._lib.tbe_evicted(self.handle, cause.ctypes.data, ids.ctypes.data, m, byref(nw)))
        return status, avail, (cause, ids)

    def acquire_batch_device(self, d_keys, d_permits, d_status, d_available, wait: bool = False,
                             id_base: int = 0, stream: Optional[int] = None) -> None:
        """Device tensors in and out; enqueued (tbe_approx_acquire_batch_device)."""
        n = d_keys.numel()
        self._check(self._lib.tbe_approx_acquire_batch_device(
            self.handle, d_keys.data_ptr(), d_permits.data_ptr(), n, 1 if wait else 0, id_base,
            d_status.data_ptr(), d_available.data_ptr(), stream))

    def collect(self, d_counts) -> None:
        """Local scores of every key into the int32 device tensor `d_counts` [n_keys]."""
        self._check(self._lib.tbe_approx_collect(self.handle, d_counts.data_ptr(), None))

    def sync(self, d_all_counts, n_clients: int, my_client: int, ts_us: int, stagger_us: int,
             stream: Optional[int] = None):
        """Replay the epoch's sync calls; returns the drain log (keys, request ids, available).
        stream=None: d_all_counts must be complete at the call (tbe_approx_sync); a stream
        handle: the replay is ordered after the work enqueued on that stream so far
        (tbe_approx_sync_stream), e.g. the collective or copy that produced the counts."""
        n = ctypes.c_uint64()
        if stream is None:
            self._check(self._lib.tbe_approx_sync(self.handle, d_all_counts.data_ptr(), n_clients, my_client,
                                                  ts_us, stagger_us, byref(n)))
        else:
            self._check(self._lib.tbe_approx_sync_stream(self.handle, d_all_counts.data_ptr(), n_clients,
                                                         my_client, ts_us, stagger_us, stream, byref(n)))
        return self._drain_log(n.value)

    def refresh(self, ts_us: int):
        """RefreshAsync as the only client of the global tier (A:412-508)."""
        n = ctypes.c_uint64()
        self._check(self._lib.tbe_approx_refresh(self.handle, ts_us, byref(n)))
        return self._drain_log(n.value)

    def _drain_log(self, m: int):
        keys = np.empty(m, dtype=np.uint64)
        ids = np.empty(m, dtype=np.int64)
        rem = np.empty(m, dtype=np.int32)
        nw = ctypes.c_uint64()
        if m:
            self._check(self._lib.tbe_refresh_log(self.handle, keys.ctypes.data, ids.ctypes.data,
                                                  rem.ctypes.data, m, byref(nw)))
        return keys, ids, rem

    def export_global(self, first: int = 0, count: Optional[int] = None):
        """Replica of the global tier (tbe_approx_export_state): (v, p, t_us), t_us =
        INT64_MIN for absent keys."""
        if count is None:
            count = self.n_keys - first
        v = np.empty(count, dtype=np.float64)
        p = np.empty(count, dtype=np.float64)
        t = np.empty(count, dtype=np.int64)
        self._check(self._lib.tbe_approx_export_state(self.handle, first, count, v.ctypes.data,
                                                      p.ctypes.data, t.ctypes.data))
        return v, p, t

    def import_global(self, v, p, t_us, first: int = 0) -> None:
        """Restore rows of the global-tier replica (tbe_approx_import_state)."""
        v = np.ascontiguousarray(v, dtype=np.float64)
        p = np.ascontiguousarray(p, dtype=np.float64)
        t_us = np.ascontiguousarray(t_us, dtype=np.int64)
        if not (v.shape == p.shape == t_us.shape):
            raise ValueError("v, p and t_us must have the same length")
        self._check(self._lib.tbe_approx_import_state(self.handle, first, v.shape[0], v.ctypes.data,
                                                      p.ctypes.data, t_us.ctypes.data))

    def local_state(self, key: int):
        """(local, global, est, available, queued) of one key."""
        lo, gl, av = c_int32(), c_int32(), c_int32()
        est = c_double()
        q = c_uint32()
        self._check(self._lib.tbe_approx_query(self.handle, key, byref(lo), byref(gl), byref(est),
                                               byref(av), byref(q)))
        return lo.value, gl.value, est.value, av.value, q.value
