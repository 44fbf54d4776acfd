"""String-key directory: ``InstanceName + resourceID`` -> dense key id.

The reference's bucket key is an exact string (``BucketId = InstanceName + resourceID``,
PartitionedRedisTokenBucketRateLimiter.cs:42); Redis compares keys byte for byte.
``StringDirectory`` keeps that mapping in HBM (include/tbe_strdir.h): whole key text in
an arena, a 64-bit hash only to pick the slot, ids by first occurrence so they never
depend on hashing.  ``HostStringDirectory`` is its host mirror (tests, reference ids).

Batches travel as Arrow-style string arrays: one uint8 byte buffer and ``n + 1`` uint64
offsets (``pack_strings``).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np

from .cluster import MASK64, scramble_walk


def _as_bytes(s) -> bytes:
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


def pack_strings(strings: Iterable) -> Tuple[np.ndarray, np.ndarray]:
    """(bytes uint8 [padded to a multiple of 8], offsets uint64 [n + 1]) of the strings
    (str is UTF-8 encoded, as .NET's string -> RedisKey conversion does)."""
    parts = [_as_bytes(s) for s in strings]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    if parts:
        offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    blob = b"".join(parts)
    buf = np.zeros(max(8, (len(blob) + 7) // 8 * 8), dtype=np.uint8)
    buf[:len(blob)] = np.frombuffer(blob, dtype=np.uint8)
    return buf, offs


class HostStringDirectory:
    """Host mirror of tbe_sdir_*: strings new to it get consecutive counters in order of
    first occurrence; id = scramble_walk(counter, capacity)."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.ids = {}
        self.overflow = False

    def assign(self, strings: Sequence) -> np.ndarray:
        keys = [_as_bytes(s) for s in strings]
        new = []
        seen = set()
        for k in keys:
            if k not in self.ids and k not in seen:
                seen.add(k)
                new.append(k)
        base = len(self.ids)
        room = max(0, self.capacity - base)
        if len(new) > room:
            self.overflow = True
        if new[:room]:
            ctr = np.arange(base, base + len(new[:room]), dtype=np.uint64)
            for k, i in zip(new[:room], scramble_walk(ctr, self.capacity).tolist()):
                self.ids[k] = i
        return self.lookup(keys)

    def lookup(self, strings: Sequence) -> np.ndarray:
        get = self.ids.get
        return np.array([get(_as_bytes(s), MASK64) for s in strings], dtype=np.uint64)

    def size(self) -> int:
        return len(self.ids)


class StringDirectory:
    """The device string directory of one limiter (prefix = its InstanceName)."""

    MODES = {"auto": 0, "full": 1, "warm": 2}

    def __init__(self, capacity: int, arena_bytes: int, prefix: str = "", device: int = -1,
                 hash_bits: int = None, mode: str = "auto"):
        """mode: the assign path (tbe_sdir_set_mode): "auto" (default), "full", "warm"."""
        import ctypes
        from . import _capi
        self._lib = _capi.load()
        p = _as_bytes(prefix)
        h = ctypes.c_void_p()
        st = self._lib.tbe_sdir_create(int(capacity), int(arena_bytes), p, len(p), device, ctypes.byref(h))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, f"tbe_sdir_create({capacity}, {arena_bytes}) failed")
        self._h = h
        self.capacity = int(capacity)
        if hash_bits is not None:
            st = self._lib.tbe_sdir_set_hash_bits(self._h, int(hash_bits))
            if st != _capi.TBE_OK:
                raise _capi.TbeError(st, "tbe_sdir_set_hash_bits failed")
        self.set_mode(mode)

    def set_mode(self, mode: str) -> None:
        from . import _capi
        st = self._lib.tbe_sdir_set_mode(self._h, self.MODES[mode])
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "tbe_sdir_set_mode failed")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tbe_sdir_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _run(self, fn, d_bytes, d_offs, n_bytes: int = None):
        import torch
        from . import _capi
        from .cluster import device_stream
        d_bytes = d_bytes.contiguous()
        d_offs = d_offs.contiguous()
        n = d_offs.numel() - 1
        ids = torch.empty(max(n, 0), dtype=torch.int64, device=d_offs.device)
        nb = d_bytes.numel() if n_bytes is None else int(n_bytes)
        st = fn(self._h, d_bytes.data_ptr(), nb, d_offs.data_ptr(), max(n, 0), ids.data_ptr(),
                device_stream(d_offs.device))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "string directory call failed")
        return ids

    def assign(self, d_bytes, d_offs, n_bytes: int = None):
        """uint8 device tensor of key text + int64 device tensor of n + 1 offsets -> int64
        ids (assigning new ones)."""
        return self._run(self._lib.tbe_sdir_assign_device, d_bytes, d_offs, n_bytes)

    def lookup(self, d_bytes, d_offs, n_bytes: int = None):
        """ids of known strings, -1 (UINT64_MAX) for others; assigns nothing."""
        return self._run(self._lib.tbe_sdir_lookup_device, d_bytes, d_offs, n_bytes)

    def assign_host(self, strings: Sequence) -> np.ndarray:
        """The host-buffer entry point (tbe_sdir_assign) on a list of strings."""
        from . import _capi
        buf, offs = pack_strings(strings)
        ids = np.empty(len(offs) - 1, dtype=np.uint64)
        n_bytes = int(offs[-1]) if len(offs) else 0
        st = self._lib.tbe_sdir_assign(self._h, buf.ctypes.data, n_bytes, offs.ctypes.data, len(offs) - 1,
                                       ids.ctypes.data)
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "tbe_sdir_assign failed")
        return ids

    def size(self) -> int:
        import ctypes
        from . import _capi
        n = ctypes.c_uint64()
        st = self._lib.tbe_sdir_size(self._h, ctypes.byref(n))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "string directory over capacity" if st == _capi.TBE_ERANGE
                                 else "string directory error")
        return n.value

    def key_of(self, key_id: int) -> bytes:
        import ctypes
        from . import _capi
        ln = ctypes.c_uint64()
        st = self._lib.tbe_sdir_key_of(self._h, int(key_id), None, 0, ctypes.byref(ln))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, f"no key with id {key_id}")
        buf = ctypes.create_string_buffer(max(1, ln.value))
        st = self._lib.tbe_sdir_key_of(self._h, int(key_id), buf, ln.value, ctypes.byref(ln))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, f"no key with id {key_id}")
        return buf.raw[:ln.value]


def to_device(strings: Sequence, device) -> Tuple["object", "object", int]:
    """(uint8 bytes tensor, int64 offsets tensor, n_bytes) of the strings on `device`."""
    import torch
    buf, offs = pack_strings(strings)
    return (torch.from_numpy(buf).to(device), torch.from_numpy(offs.view(np.int64)).to(device),
            int(offs[-1]) if len(offs) else 0)


def synthetic_key_text(d_keys, prefix: str = "resource-"):
    """Device key text prefix + decimal(key) for an int64 device tensor of keys
    (tbe_key_text_*, benchmark and tests): (uint8 bytes, int64 offsets [n + 1], n_bytes)."""
    import torch
    from . import _capi
    from .cluster import device_stream
    lib = _capi.load()
    dev = d_keys.device
    st = device_stream(dev)
    d_keys = d_keys.contiguous()
    n = d_keys.numel()
    p = _as_bytes(prefix)
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    if lib.tbe_key_text_lengths_device(d_keys.data_ptr(), n, len(p), lens.data_ptr(), st) != 0:
        raise RuntimeError("tbe_key_text_lengths_device failed")
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    n_bytes = int(offs[-1].item()) if n else 0
    buf = torch.empty((n_bytes + 7) // 8 * 8 + 8, dtype=torch.uint8, device=dev)
    if lib.tbe_key_text_device(d_keys.data_ptr(), n, p, len(p), offs.data_ptr(), buf.data_ptr(), st) != 0:
        raise RuntimeError("tbe_key_text_device failed")
    return buf, offs, n_bytes


__all__: List[str] = ["pack_strings", "HostStringDirectory", "StringDirectory", "to_device", "synthetic_key_text"]
