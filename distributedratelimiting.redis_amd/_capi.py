"""ctypes binding of ``include/tbe.h`` (the engine's C ABI).

This is the same surface a .NET host would P/Invoke.  Loading fails
loudly when ``libtbe.so`` has not been built: there is no CPU fallback anywhere in
the product path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_int32, c_int64, c_uint8,
                    c_uint32, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtbe.so")

TBE_OK, TBE_EINVAL, TBE_ENOMEM, TBE_EDEVICE, TBE_EDISPOSED, TBE_ERANGE = range(6)
STATUS_NAMES = {0: "TBE_OK", 1: "TBE_EINVAL", 2: "TBE_ENOMEM", 3: "TBE_EDEVICE",
                4: "TBE_EDISPOSED", 5: "TBE_ERANGE"}
TBE_KIND_TOKEN_BUCKET, TBE_KIND_QUEUEING, TBE_KIND_APPROXIMATE = 0, 1, 2
TBE_FLAG_STAGE_TIMING = 0x1
TBE_FLAG_FOLD_TIMING = 0x100
TBE_FLAG_NO_PACK = 0x2
TBE_FLAG_NO_HOT = 0x4
TBE_FLAG_NO_PIPELINE = 0x8
TBE_FLAG_NO_NARROW = 0x10
TBE_FLAG_UNSCATTER_ALL = 0x20
TBE_FLAG_HIST_RECORDS = 0x40
TBE_FLAG_RERANK = 0x80
STAGES = ("hist", "colscan", "scatter", "bounds", "fold", "unscatter", "hot")

# Every symbol include/tbe.h declares (tests/test_capi_symbols.py checks the header too).
EXPORTED = ("tbe_fill_rate", "tbe_create", "tbe_destroy", "tbe_last_error", "tbe_acquire_batch",
            "tbe_acquire_batch_device", "tbe_synchronize", "tbe_query", "tbe_export_state",
            "tbe_wait_batch", "tbe_queue_attempt_batch", "tbe_evicted", "tbe_refresh", "tbe_refresh_log", "tbe_queue_of",
            "tbe_approx_acquire_batch", "tbe_approx_collect", "tbe_approx_sync", "tbe_approx_refresh",
            "tbe_approx_query", "tbe_layout", "tbe_stage_times", "tbe_wait_batch_device",
            "tbe_refresh_bound", "tbe_refresh_device", "tbe_approx_acquire_batch_device",
            "tbe_import_state", "tbe_queue_cancel", "tbe_alloc_host", "tbe_free_host",
            "tbe_approx_export_state", "tbe_approx_import_state", "tbe_wait_batch_tick_device",
            "tbe_approx_sync_stream", "tbe_batch_format")
TBE_WAIT_FAILED, TBE_WAIT_GRANTED, TBE_WAIT_QUEUED, TBE_WAIT_REJECTED = 0, 1, 2, 3


class TbeConfig(Structure):
    _fields_ = [
        ("struct_size", c_uint32),
        ("kind", c_int32),
        ("n_keys", c_uint64),
        ("token_limit", c_int32),
        ("tokens_per_period", c_int32),
        ("replenishment_period_ticks", c_int64),
        ("queue_limit", c_int32),
        ("queue_order", c_int32),
        ("device", c_int32),
        ("flags", c_uint32),
        ("max_batch", c_uint64),
        ("zero_wait_slots", c_int32),
        ("reserved", c_int32),
    ]


class TbeError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


_lib = None


def load(path: str = None) -> ctypes.CDLL:
    """Load libtbe.so (once).  Raises FileNotFoundError if it was never built.
    ``TBE_LIB`` overrides the path (ablation builds in tools/ only)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("TBE_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} is missing: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    lib.tbe_fill_rate.restype = c_double
    lib.tbe_fill_rate.argtypes = [c_int32, c_int64]
    lib.tbe_create.restype = c_int32
    lib.tbe_create.argtypes = [POINTER(TbeConfig), POINTER(c_void_p)]
    lib.tbe_destroy.restype = None
    lib.tbe_destroy.argtypes = [c_void_p]
    lib.tbe_last_error.restype = c_char_p
    lib.tbe_last_error.argtypes = [c_void_p]
    lib.tbe_acquire_batch.restype = c_int32
    lib.tbe_acquire_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                      c_void_p]
    lib.tbe_acquire_batch_device.restype = c_int32
    lib.tbe_acquire_batch_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64,
                                             c_void_p, c_void_p, c_void_p]
    lib.tbe_synchronize.restype = c_int32
    lib.tbe_synchronize.argtypes = [c_void_p]
    lib.tbe_query.restype = c_int32
    lib.tbe_query.argtypes = [c_void_p, c_uint64, c_int64, POINTER(c_double), POINTER(c_double),
                              POINTER(c_int32)]
    lib.tbe_export_state.restype = c_int32
    lib.tbe_export_state.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]
    lib.tbe_wait_batch.restype = c_int32
    lib.tbe_wait_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int64, c_void_p,
                                   c_void_p, POINTER(c_uint64)]
    lib.tbe_evicted.restype = c_int32
    lib.tbe_evicted.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]
    lib.tbe_refresh.restype = c_int32
    lib.tbe_refresh.argtypes = [c_void_p, c_int64, POINTER(c_uint64)]
    lib.tbe_refresh_log.restype = c_int32
    lib.tbe_refresh_log.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]
    lib.tbe_queue_of.restype = c_int32
    lib.tbe_queue_of.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, POINTER(c_uint32)]
    lib.tbe_alloc_host.restype = c_int32
    lib.tbe_alloc_host.argtypes = [c_uint64, POINTER(c_void_p)]
    lib.tbe_free_host.restype = None
    lib.tbe_free_host.argtypes = [c_void_p]
    lib.tbe_queue_cancel.restype = c_int32
    lib.tbe_queue_cancel.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, POINTER(c_uint64)]
    lib.tbe_approx_acquire_batch.restype = c_int32
    lib.tbe_approx_acquire_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_int32, c_int64,
                                             c_void_p, c_void_p, POINTER(c_uint64)]
    lib.tbe_approx_collect.restype = c_int32
    lib.tbe_approx_collect.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.tbe_approx_sync.restype = c_int32
    lib.tbe_approx_sync.argtypes = [c_void_p, c_void_p, c_uint32, c_uint32, c_int64, c_int64,
                                    POINTER(c_uint64)]
    lib.tbe_batch_format.restype = c_int32
    lib.tbe_batch_format.argtypes = [c_void_p, c_uint64, c_void_p, c_uint32]
    lib.tbe_approx_sync_stream.restype = c_int32
    lib.tbe_approx_sync_stream.argtypes = [c_void_p, c_void_p, c_uint32, c_uint32, c_int64, c_int64, c_void_p,
                                           POINTER(c_uint64)]
    lib.tbe_queue_attempt_batch.restype = c_int32
    lib.tbe_queue_attempt_batch.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                            c_void_p]
    lib.tbe_approx_refresh.restype = c_int32
    lib.tbe_approx_refresh.argtypes = [c_void_p, c_int64, POINTER(c_uint64)]
    lib.tbe_approx_query.restype = c_int32
    lib.tbe_approx_query.argtypes = [c_void_p, c_uint64, POINTER(c_int32), POINTER(c_int32),
                                     POINTER(c_double), POINTER(c_int32), POINTER(c_uint32)]
    lib.tbe_wait_batch_device.restype = c_int32
    lib.tbe_wait_batch_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int64,
                                          c_int32, c_void_p, c_void_p, c_void_p]
    lib.tbe_refresh_bound.restype = c_int32
    lib.tbe_refresh_bound.argtypes = [c_void_p, POINTER(c_uint64)]
    lib.tbe_refresh_device.restype = c_int32
    lib.tbe_refresh_device.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_uint64,
                                       c_void_p, c_void_p]
    lib.tbe_wait_batch_tick_device.restype = c_int32
    lib.tbe_wait_batch_tick_device.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int64,
                                               c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                               c_void_p, c_uint64, c_void_p, c_void_p]
    lib.tbe_approx_acquire_batch_device.restype = c_int32
    lib.tbe_approx_acquire_batch_device.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_int32,
                                                    c_int64, c_void_p, c_void_p, c_void_p]
    lib.tbe_import_state.restype = c_int32
    lib.tbe_import_state.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]
    lib.tbe_approx_export_state.restype = c_int32
    lib.tbe_approx_export_state.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]
    lib.tbe_approx_import_state.restype = c_int32
    lib.tbe_approx_import_state.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p]
    lib.tbe_gen_zipf_keys_device.restype = c_int32
    lib.tbe_gen_zipf_keys_device.argtypes = [c_uint64, c_uint64, c_double, c_uint64, c_uint64, c_void_p,
                                             c_void_p]
    lib.tbe_gen_batch_device.restype = c_int32
    lib.tbe_gen_batch_device.argtypes = [c_uint64] * 4 + [c_int32] * 2 + [c_int64] * 2 + [c_void_p] * 4
    # multi-GPU path (include/tbe_cluster.h)
    lib.tbe_key_owner.restype = c_uint32
    lib.tbe_key_owner.argtypes = [c_uint64, c_uint32]
    lib.tbe_route_workspace_bytes.restype = c_uint64
    lib.tbe_route_workspace_bytes.argtypes = [c_uint64, c_uint32]
    lib.tbe_route_plan_device.restype = c_int32
    lib.tbe_route_plan_device.argtypes = [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.tbe_route_plan_map_device.restype = c_int32
    lib.tbe_route_plan_map_device.argtypes = [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p]
    lib.tbe_key_vnode.restype = c_uint32
    lib.tbe_key_vnode.argtypes = [c_uint64]
    lib.tbe_vnode_count_device.restype = c_int32
    lib.tbe_vnode_count_device.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p]
    lib.tbe_route_pack_device.restype = c_int32
    lib.tbe_route_pack_device.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.tbe_route_gather_device.restype = c_int32
    lib.tbe_route_gather_device.argtypes = [c_void_p, c_uint64, c_void_p, c_uint32, c_void_p, c_void_p]
    lib.tbe_dir_create.restype = c_int32
    lib.tbe_dir_create.argtypes = [c_uint64, c_int32, POINTER(c_void_p)]
    lib.tbe_dir_destroy.restype = None
    lib.tbe_dir_destroy.argtypes = [c_void_p]
    lib.tbe_dir_assign_device.restype = c_int32
    lib.tbe_dir_assign_device.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]
    lib.tbe_dir_lookup_device.restype = c_int32
    lib.tbe_dir_lookup_device.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]
    lib.tbe_dir_size.restype = c_int32
    lib.tbe_dir_size.argtypes = [c_void_p, POINTER(c_uint64)]
    lib.tbe_dir_state_async.restype = c_int32
    lib.tbe_dir_state_async.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.tbe_key_text_lengths_device.restype = c_int32
    lib.tbe_key_text_lengths_device.argtypes = [c_void_p, c_uint64, ctypes.c_uint32, c_void_p, c_void_p]
    lib.tbe_key_text_device.restype = c_int32
    lib.tbe_key_text_device.argtypes = [c_void_p, c_uint64, ctypes.c_char_p, ctypes.c_uint32, c_void_p, c_void_p,
                                        c_void_p]
    # string-key directory (include/tbe_strdir.h)
    lib.tbe_sdir_create.restype = c_int32
    lib.tbe_sdir_create.argtypes = [c_uint64, c_uint64, ctypes.c_char_p, ctypes.c_uint32, c_int32, POINTER(c_void_p)]
    lib.tbe_sdir_destroy.restype = None
    lib.tbe_sdir_destroy.argtypes = [c_void_p]
    for fn in ("tbe_sdir_assign_device", "tbe_sdir_lookup_device"):
        getattr(lib, fn).restype = c_int32
        getattr(lib, fn).argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, c_void_p]
    lib.tbe_sdir_assign.restype = c_int32
    lib.tbe_sdir_assign.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_void_p]
    lib.tbe_sdir_size.restype = c_int32
    lib.tbe_sdir_size.argtypes = [c_void_p, POINTER(c_uint64)]
    lib.tbe_sdir_key_of.restype = c_int32
    lib.tbe_sdir_key_of.argtypes = [c_void_p, c_uint64, c_void_p, c_uint64, POINTER(c_uint64)]
    lib.tbe_sdir_set_hash_bits.restype = c_int32
    lib.tbe_sdir_set_hash_bits.argtypes = [c_void_p, ctypes.c_uint32]
    lib.tbe_sdir_set_mode.restype = c_int32
    lib.tbe_sdir_set_mode.argtypes = [c_void_p, c_int32]
    lib.tbe_numfmt_device.restype = c_int32
    lib.tbe_numfmt_device.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p]
    lib.tbe_layout.restype = c_int32
    lib.tbe_layout.argtypes = [c_void_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]
    lib.tbe_stage_times.restype = c_int32
    lib.tbe_stage_times.argtypes = [c_void_p, POINTER(c_double), c_uint32, POINTER(c_uint32)]
    _lib = lib
    return lib


def make_config(n_keys: int, token_limit: int, tokens_per_period: int, period_ticks: int,
                kind: int = TBE_KIND_TOKEN_BUCKET, queue_limit: int = 0, queue_order: int = 0,
                device: int = -1, flags: int = 0, max_batch: int = 0,
                zero_wait_slots: int = 0) -> TbeConfig:
    return TbeConfig(ctypes.sizeof(TbeConfig), kind, n_keys, token_limit, tokens_per_period,
                     period_ticks, queue_limit, queue_order, device, flags, max_batch,
                     zero_wait_slots, 0)
