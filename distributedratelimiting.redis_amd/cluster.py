"""Multi-GPU layer: one engine per GPU (one process per rank), keys hash-partitioned.

The reference distributes by letting many client processes share one Redis key space
(the bucket key is ``InstanceName + resourceID``, PTB:42).  Here every key
has exactly one owner GPU holding its bucket state:

    owner(key) = ((mix64(key) >> 32) * world) >> 32      (= mix64(key) >> (64 - log2 world))

or, with an owner map (every routing call takes ``owner_map=``), the map's entry for the
key's virtual node (the top 12 bits of mix64(key)): ``balanced_owner_map`` builds one from
observed per-virtual-node loads so that a Zipf stream's hot keys do not overload their
owners, and the owner's key directory (``tbe_dir_*``, device-resident and collision-free: it
stores whole keys) turns the keys it owns into dense bucket ids.  The token-bucket paths
need no collective when ingest is already partitioned (the benchmark's default mode).
Exchanges:

* ``route_requests`` / ``route_replies`` (``route_batch`` = both around a ``decide``):
  requests that arrive at any rank travel to their owner in one all-to-all (grouped by a
  stable partition, so a key's requests reach the owner in (source rank, arrival) order,
  a valid serial order of the reference) and the replies come back in a reverse
  all-to-all.  On GPUs everything stays in HBM (``tbe_route_*`` kernels + RCCL); only the
  world group sizes go through the host, as the all-to-all's split sizes.
* ``route_cancel``: cancellations of queued requests travel to the key's owner the same
  way (one all-to-all each way).
* ``approx_epoch``: the ApproximateTokenBucket global tier.  Each rank is one client
  (A:9-599) holding a local tier for every shared key; at every refresh epoch the
  per-key consumed counts are exchanged -- all-gather for exact per-client prefix
  semantics (client r's sync call sees clients 0..r-1, SURVEY.md §8e option 2), or
  all-reduce when the node acts as ONE client (option 1) -- and every rank replays the
  same sync calls on its replica of the global tier.

Inputs as CUDA tensors take the device path (backend "nccl" = RCCL over xGMI); numpy
arrays take a host path with identical semantics (backend "gloo", the CPU tests).  The
device path also runs over a "gloo" group (its collectives then stage through host
memory): that is how two ranks sharing one GPU exercise the whole device path in the
tests (RCCL refuses two ranks on one device).

Directories never free ids (a key keeps its bucket for the directory's lifetime, like a
Redis key that has not expired); a batch that brings more new keys than ids remain
raises ``TbeError(TBE_ERANGE)`` before any decision is made, and the directory must be
recreated.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1
NO_ID = np.uint64(MASK64)


# ------------------------------------------------------------------ key partitioning
def _mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z *= np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return z


def key_owner(keys, world: int, owner_map=None) -> np.ndarray:
    """Owner rank of each key (csrc/tbe_hash.hpp key_owner): ((mix64(key) >> 32) * world)
    >> 32, i.e. the top log2(world) bits of mix64(key) for a power-of-two world; with an
    owner map (include/tbe_cluster.h), owner_map[key_vnode(key)]."""
    if owner_map is not None:
        return np.asarray(check_owner_map(owner_map, world), dtype=np.int64)[key_vnode(keys)]
    h = _mix64(keys) >> np.uint64(32)
    with np.errstate(over="ignore"):
        return ((h * np.uint64(world)) >> np.uint64(32)).astype(np.int64)


# ------------------------------------------------------------------ owner maps
OWNER_MAP_BITS = 12                  # include/tbe_cluster.h TBE_OWNER_MAP_BITS
OWNER_MAP_SIZE = 1 << OWNER_MAP_BITS


def key_vnode(keys) -> np.ndarray:
    """Virtual node of each key: the top 12 bits of mix64(key) (tbe_key_vnode)."""
    return (_mix64(keys) >> np.uint64(64 - OWNER_MAP_BITS)).astype(np.int64)


def check_owner_map(owner_map, world: int):
    """Validate an owner map before any kernel reads it (include/tbe_cluster.h: a u8 array
    of exactly 4096 entries, each < world).  A CUDA tensor's shape and dtype are checked
    here; its values are not read back (that would synchronise every routed batch) -- the
    route kernels clamp an entry >= world to world - 1, so a bad device map misroutes but
    never writes out of bounds.  Returns the map unchanged; raises ValueError otherwise."""
    if _is_cuda(owner_map):
        import torch
        if owner_map.dtype != torch.uint8 or owner_map.numel() != OWNER_MAP_SIZE:
            raise ValueError(f"owner map must be {OWNER_MAP_SIZE} uint8 entries")
        return owner_map
    m = np.asarray(owner_map)
    if m.shape != (OWNER_MAP_SIZE,):
        raise ValueError(f"owner map must have exactly {OWNER_MAP_SIZE} entries, got shape {m.shape}")
    if m.dtype != np.uint8:
        if not np.issubdtype(m.dtype, np.integer) or m.min() < 0 or m.max() > 255:
            raise ValueError("owner map entries must be uint8 owner ranks")
    if int(m.max()) >= world:
        raise ValueError(f"owner map entry {int(m.max())} >= world ({world})")
    return m


def hash_owner_map(world: int) -> np.ndarray:
    """The owner map equal to the hash partition for a power-of-two world:
    v -> (v * world) >> 12."""
    if world & (world - 1) or not 1 <= world <= OWNER_MAP_SIZE:
        raise ValueError("the hash owner map needs a power-of-two world <= 4096")
    return ((np.arange(OWNER_MAP_SIZE, dtype=np.int64) * world) >> OWNER_MAP_BITS).astype(np.uint8)


# Keys one engine holds in its fastest layout: two 8-bit LSD passes over the bucket ids
# (2^11 keys per bucket) with room for the 1024 hot-key buckets, and packed 8-byte records.
# Past it the engine takes a third partition pass, and past 2^27 keys its records no longer
# pack (a 28-bit key field leaves under 32 bits for the time offset), which also turns off
# hot-key runs: on Zipf traffic that is a cliff, not a slope (DESIGN.md §7 "owner maps").
PACKED_KEYS_MAX = (65536 - 1024) << 11


def max_vnodes_per_owner(n_keys: int, world: int, slack: float = 0.01, limit: int = PACKED_KEYS_MAX) -> int:
    """The most virtual nodes one owner may take while its table (keys_per_rank) stays
    within `limit` keys; never fewer than the even share ceil(4096 / world)."""
    fair = -(-OWNER_MAP_SIZE // world)
    best = fair
    for m in range(fair + 1, OWNER_MAP_SIZE + 1):
        share = -(-n_keys * m // OWNER_MAP_SIZE)
        if min(n_keys, int(share * (1.0 + slack)) + 1024) > limit:
            break
        best = m
    return best


def balanced_owner_map(loads, world: int, n_keys: int | None = None) -> np.ndarray:
    """An owner map that evens out the owners' request loads (DESIGN.md §7 "owner maps").
    loads[v] = requests observed on virtual node v (e.g. all ranks' vnode counts of a
    batch, all-reduced so that every rank builds the same map).  Longest processing time
    first: virtual nodes by descending load (ties by index), each to the owner with the
    least load so far (ties to the lowest rank), virtual nodes without load spread so that
    every owner ends with about the same number of them (its share of the key space).
    n_keys (the global key space): no owner takes more than max_vnodes_per_owner virtual
    nodes, so every owner's table stays in the packed two-pass layout -- the owner of a
    very hot key then keeps more of the load than the others instead of pushing their
    tables over that limit.  Deterministic: the same loads give the same map on every rank."""
    loads = np.asarray(loads, dtype=np.int64).reshape(-1)
    if loads.size != OWNER_MAP_SIZE or world < 1 or world > 256:
        raise ValueError("loads must have 4096 entries and 1 <= world <= 256")
    order = np.lexsort((np.arange(OWNER_MAP_SIZE), -loads))
    out = np.empty(OWNER_MAP_SIZE, dtype=np.uint8)
    acc = np.zeros(world, dtype=np.int64)
    nv = np.zeros(world, dtype=np.int64)
    cap_v = -(-OWNER_MAP_SIZE // world)
    cap = OWNER_MAP_SIZE if n_keys is None else max_vnodes_per_owner(n_keys, world)
    big = np.iinfo(np.int64).max
    for v in order.tolist():
        if loads[v] > 0:
            r = int(np.argmin(np.where(nv < cap, acc, big)))
        else:   # no load seen: keep the owners' shares of the key space level
            r = int(np.argmin(np.where(nv < cap_v, nv, OWNER_MAP_SIZE + 1)))
        out[v] = r
        acc[r] += loads[v]
        nv[r] += 1
    return out


def _scramble_params(n: int):
    bits = max(1, int(n - 1).bit_length())
    return np.uint64((1 << bits) - 1), np.uint64(max(1, bits // 2))


def _scramble(x: np.ndarray, mask, sh) -> np.ndarray:
    with np.errstate(over="ignore"):
        for a, c in ((0x9E3779B97F4A7C15, 0x632BE59BD9B4E019),
                     (0xD1B54A32D192ED03, 0x8CB92BA72F3D8DD7),
                     (0xAEF17502108EF2D9, 0x2545F4914F6CDD1D)):
            x = (x * np.uint64(a) + np.uint64(c)) & mask
            x ^= x >> sh
    return x


def scramble_walk(x, n: int) -> np.ndarray:
    """The fixed bijection of [0, n) the directory applies to its counters
    (csrc/tbe_hash.hpp scramble_walk)."""
    mask, sh = _scramble_params(n)
    x = _scramble(np.asarray(x, dtype=np.uint64), mask, sh)
    bad = x >= np.uint64(n)
    while bad.any():
        x[bad] = _scramble(x[bad], mask, sh)
        bad = x >= np.uint64(n)
    return x


class HostDirectory:
    """Host mirror of the device key directory (tbe_dir_*): keys new to it get counters in
    order of first occurrence, id = scramble_walk(counter, capacity).  Used by the gloo
    path and the tests."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.ids = {}
        self.overflow = False

    def check(self) -> None:
        """Raise TbeError(TBE_ERANGE) once a batch has brought more new keys than ids remained."""
        if self.overflow:
            from . import _capi
            raise _capi.TbeError(_capi.TBE_ERANGE, f"key directory over capacity ({self.capacity} ids)")

    def assign(self, keys) -> np.ndarray:
        keys = np.asarray(keys, dtype=np.uint64)
        if keys.size == 0:
            return np.zeros(0, dtype=np.uint64)
        uniq, first = np.unique(keys, return_index=True)
        new = [(f, k) for k, f in zip(uniq.tolist(), first.tolist()) if k not in self.ids]
        new.sort()
        base = len(self.ids)
        room = max(0, self.capacity - base)
        if len(new) > room:
            self.overflow = True
        if new[:room]:
            ctr = np.arange(base, base + len(new[:room]), dtype=np.uint64)
            for (_, k), i in zip(new[:room], scramble_walk(ctr, self.capacity).tolist()):
                self.ids[k] = i
        return self.lookup(keys)

    def lookup(self, keys) -> np.ndarray:
        get = self.ids.get
        return np.array([get(k, MASK64) for k in np.asarray(keys, dtype=np.uint64).tolist()], dtype=np.uint64)

    def size(self) -> int:
        return len(self.ids)


class DeviceDirectory:
    """The owner's key directory in HBM (include/tbe_cluster.h tbe_dir_*).

    ``strict`` (default): ``check()`` raises TBE_ERANGE for the very batch that overflowed,
    before anything is decided -- near capacity that costs a device synchronisation per
    batch.  ``strict=False``: near capacity each check enqueues an asynchronous copy of the
    directory's state (tbe_dir_state_async) and inspects the previous one, so an overflow
    raises one batch later without synchronising; the overflowing batch itself is still
    refused, by the engine (its keys beyond capacity get UINT64_MAX ids, an invalid batch:
    TBE_EINVAL at the engine's next synchronisation, and that batch's reply buffers are left
    unwritten).  Once an overflow has been seen every later check() raises, as in strict mode.
    bench.py --route timed uses it, so no synchronisation sits inside a timed step."""

    def __init__(self, capacity: int, device: int = -1, strict: bool = True):
        import ctypes
        from . import _capi
        self._lib = _capi.load()
        h = ctypes.c_void_p()
        st = self._lib.tbe_dir_create(int(capacity), device, ctypes.byref(h))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, f"tbe_dir_create({capacity}) failed")
        self._h = h
        self.capacity = int(capacity)
        # upper bound of the ids assigned so far (each key of an assign batch adds at most
        # one): while it stays below capacity no batch can have overflowed, so the exact
        # count (a device synchronisation) is fetched only once the bound reaches it
        self._bound = 0
        self.strict = strict
        self._pending = None     # (pinned state copy, event) of the last asynchronous check
        self._overflowed = False  # an asynchronous check saw the (sticky) overflow bit

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.tbe_dir_destroy(self._h)
            self._h = None

    def check(self) -> None:
        """Raise TbeError(TBE_ERANGE) if an assign batch overflowed the directory; free
        (no device synchronisation) while the assigned-id bound stays below capacity."""
        if self._bound < self.capacity:
            return
        if self.strict:
            self._bound = self.size()      # raises TBE_ERANGE on overflow
            return
        import torch
        from . import _capi
        if self._overflowed:   # the overflow bit is sticky: refuse every later batch too
            raise _capi.TbeError(_capi.TBE_ERANGE, f"key directory over capacity ({self.capacity} ids)")
        if self._pending is not None and self._pending[1].query():
            st = self._pending[0]
            self._pending = None
            if int(st[1]) != 0:
                self._overflowed = True
                raise _capi.TbeError(_capi.TBE_ERANGE, f"key directory over capacity ({self.capacity} ids)")
        if self._pending is None:
            dev = torch.device("cuda", torch.cuda.current_device())
            st = torch.zeros(2, dtype=torch.int64, pin_memory=True)
            rc = self._lib.tbe_dir_state_async(self._h, st.data_ptr(), device_stream(dev))
            if rc != _capi.TBE_OK:
                raise _capi.TbeError(rc, "tbe_dir_state_async failed")
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._pending = (st, ev)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _run(self, fn, d_keys):
        import torch
        from . import _capi
        if not _is_cuda(d_keys) or d_keys.dtype not in (torch.int64, torch.uint64):
            raise TypeError("DeviceDirectory takes an int64 (or uint64) CUDA tensor of keys")
        d_keys = d_keys.contiguous()
        ids = torch.empty(d_keys.numel(), dtype=torch.int64, device=d_keys.device)
        st = fn(self._h, d_keys.data_ptr(), d_keys.numel(), ids.data_ptr(), device_stream(d_keys.device))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "directory call failed")
        return ids

    def assign(self, d_keys):
        """int64 device tensor of keys -> int64 device tensor of ids (assigning new ones;
        keys beyond capacity get -1, and check() raises from then on)."""
        ids = self._run(self._lib.tbe_dir_assign_device, d_keys)
        self._bound += d_keys.numel()
        return ids

    def lookup(self, d_keys):
        """ids of known keys, -1 (UINT64_MAX) for others; assigns nothing."""
        return self._run(self._lib.tbe_dir_lookup_device, d_keys)

    def size(self) -> int:
        import ctypes
        from . import _capi
        n = ctypes.c_uint64()
        st = self._lib.tbe_dir_size(self._h, ctypes.byref(n))
        if st != _capi.TBE_OK:
            raise _capi.TbeError(st, "directory over capacity" if st == _capi.TBE_ERANGE else "tbe_dir_size failed")
        return n.value


def keys_per_rank(n_keys: int, world: int, slack: float = 0.01, owner_map=None) -> int:
    """Table capacity per rank for n_keys hash-partitioned keys: the expected share plus
    a margin far above the binomial spread of the owner counts.  With an owner map, the
    share of the owner with the most virtual nodes (each holds 1/4096 of the keys)."""
    if world == 1:
        return n_keys
    if owner_map is not None:
        most = int(np.bincount(np.asarray(owner_map, dtype=np.int64), minlength=world).max())
        share = -(-n_keys * most // OWNER_MAP_SIZE)
    else:
        share = -(-n_keys // world)
    return min(n_keys, int(share * (1.0 + slack)) + 1024)


def vnode_loads(d_keys):
    """Requests per virtual node of a device batch (tbe_vnode_count_device): int64 [4096]."""
    import torch
    from . import _capi
    lib = _capi.load()
    d_keys = _device_columns(d_keys)[0]
    out = torch.empty(OWNER_MAP_SIZE, dtype=torch.int64, device=d_keys.device)
    _check(lib.tbe_vnode_count_device(d_keys.data_ptr(), d_keys.numel(), out.data_ptr(), device_stream(d_keys.device)))
    return out


def _device_map(owner_map, dev, world: int):
    """The owner map as a u8 device tensor (NULL pointer for the hash partition), validated
    (check_owner_map) so that no route kernel sees an entry >= world."""
    if owner_map is None:
        return None
    import torch
    check_owner_map(owner_map, world)
    m = owner_map if _is_cuda(owner_map) else torch.from_numpy(np.ascontiguousarray(owner_map, dtype=np.uint8))
    return m.to(device=dev, dtype=torch.uint8).contiguous()


# ------------------------------------------------------------------ collectives
def _stages_through_host(t, group) -> bool:
    """A CUDA tensor on a gloo group: gloo's all-to-all / all-gather take host tensors."""
    import torch.distributed as dist
    return _is_cuda(t) and dist.get_backend(group) == "gloo"


def _all_to_all(out, inp, out_splits=None, in_splits=None, group=None) -> None:
    import torch.distributed as dist
    if _stages_through_host(inp, group):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)


def _all_gather(out, inp, group=None) -> None:
    import torch.distributed as dist
    if _stages_through_host(inp, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
        return
    dist.all_gather_into_tensor(out, inp, group=group)


def _all_reduce_sum(t, group=None) -> None:
    import torch.distributed as dist
    if _stages_through_host(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
        return
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


# ------------------------------------------------------------------ all-to-all routing
class RoutePlan:
    """What route_replies needs to send replies back: the arrival -> grouped permutation
    and the all-to-all split sizes of both directions."""

    def __init__(self, order, send_counts, recv_counts, n):
        self.order, self.send_counts, self.recv_counts, self.n = order, send_counts, recv_counts, n


def _is_cuda(x) -> bool:
    return hasattr(x, "is_cuda") and x.is_cuda


def route_requests(keys, permits, ts_us, directory, group=None, owner_map=None):
    """Send this rank's requests to their owners.  Returns ((local ids, permits, ts) of
    the requests this rank owns, in (source rank, arrival) order, and the RoutePlan for
    route_replies).  CUDA tensors: device kernels + RCCL; numpy: host path + gloo.
    owner_map: table-driven ownership (balanced_owner_map), the same on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if _is_cuda(keys):
        dev = keys.device
        keys, permits, ts_us = _device_columns(keys, (permits, torch.int32), (ts_us, torch.int64))
        pos, sc_l, rc_l, recv = _route_device(keys, permits, ts_us, world, group, owner_map)
        local = directory.assign(recv[:, 0])
        directory.check()        # an over-capacity batch raises before anything is decided
        return (local, recv[:, 2].to(torch.int32), recv[:, 1].contiguous()), RoutePlan(pos, sc_l, rc_l, keys.numel())
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.shape[0]
    owner = key_owner(keys, world, owner_map)
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    sc = torch.from_numpy(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = rc.numpy()
    payload = np.stack([keys[order].view(np.int64), np.asarray(ts_us, dtype=np.int64)[order],
                        np.asarray(permits, dtype=np.int64)[order]], axis=1)
    recv = torch.empty((int(recv_counts.sum()), 3), dtype=torch.int64)
    dist.all_to_all_single(recv, torch.from_numpy(np.ascontiguousarray(payload)),
                           output_split_sizes=recv_counts.tolist(), input_split_sizes=send_counts.tolist(),
                           group=group)
    r = recv.numpy()
    local = directory.assign(r[:, 0].view(np.uint64))
    directory.check()
    return (local, r[:, 2].astype(np.int32), r[:, 1].copy()), RoutePlan(order, send_counts.tolist(),
                                                                        recv_counts.tolist(), n)


def _device_columns(keys, *cols):
    """The device path's input contract: keys int64 (uint64 is reinterpreted), the other
    columns converted to the dtype the route kernels read, all on the keys' device."""
    import torch
    if keys.dtype == torch.uint64:
        keys = keys.view(torch.int64)
    if keys.dtype != torch.int64:
        raise TypeError(f"keys must be an int64 or uint64 tensor, not {keys.dtype}")
    out = [keys.contiguous()]
    for c, dt in cols:
        if not _is_cuda(c) or c.device != keys.device:
            raise ValueError("every column of a device-path batch must be on the keys' device")
        if c.numel() != keys.numel():
            raise ValueError("columns differ in length")
        out.append(c.to(dt).contiguous())
    return tuple(out)


def _route_device(keys, permits, payload, world, group, owner_map=None):
    """Owner-grouped exchange of {key, payload i64, permits i32} records on the device:
    tbe_route_plan_map_device + tbe_route_pack_device, the split sizes by all-to-all, the
    records by all-to-all.  Returns (pos, send counts, recv counts, recv [m, 3] int64)."""
    import torch
    from . import _capi
    lib = _capi.load()
    dev = keys.device
    stream = device_stream(dev)
    n = keys.numel()
    pos = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    counts = torch.zeros(world, dtype=torch.int64, device=dev)
    work = torch.empty(max(1, lib.tbe_route_workspace_bytes(n, world)), dtype=torch.uint8, device=dev)
    dmap = _device_map(owner_map, dev, world)
    _check(lib.tbe_route_plan_map_device(keys.data_ptr(), n, world, dmap.data_ptr() if dmap is not None else None,
                                         work.data_ptr(), pos.data_ptr(), counts.data_ptr(), stream))
    send = torch.empty((n, 3), dtype=torch.int64, device=dev)
    _check(lib.tbe_route_pack_device(pos.data_ptr(), n, keys.data_ptr(), permits.data_ptr(),
                                     payload.data_ptr(), send.data_ptr(), stream))
    rc = torch.empty_like(counts)
    _all_to_all(rc, counts, group=group)
    sc_l, rc_l = counts.tolist(), rc.tolist()
    recv = torch.empty((sum(rc_l), 3), dtype=torch.int64, device=dev)
    _all_to_all(recv, send, rc_l, sc_l, group=group)
    return pos, sc_l, rc_l, recv


def route_replies(plan: RoutePlan, cols, group=None):
    """Send the owner's reply columns (one int64-convertible array/tensor per column, in
    route_requests' received order) back; returns them in this rank's arrival order."""
    import torch
    import torch.distributed as dist

    if cols and _is_cuda(cols[0]):
        from . import _capi
        lib = _capi.load()
        dev = cols[0].device
        reply = torch.stack([c.to(torch.int64) for c in cols], dim=1).contiguous()
        k = reply.shape[1]
        back = torch.empty((plan.n, k), dtype=torch.int64, device=dev)
        _all_to_all(back, reply, plan.send_counts, plan.recv_counts, group=group)
        out = torch.empty_like(back)
        _check(lib.tbe_route_gather_device(plan.order.data_ptr(), plan.n, back.data_ptr(), k, out.data_ptr(),
                                           device_stream(dev)))
        return tuple(out[:, c] for c in range(k))
    k = len(cols)
    m = sum(plan.recv_counts)
    reply = np.stack([np.asarray(c, dtype=np.int64).reshape(-1) for c in cols], axis=1) if m \
        else np.zeros((0, k), dtype=np.int64)
    back = torch.empty((plan.n, k), dtype=torch.int64)
    dist.all_to_all_single(back, torch.from_numpy(np.ascontiguousarray(reply)),
                           output_split_sizes=plan.send_counts, input_split_sizes=plan.recv_counts, group=group)
    b = back.numpy()
    out = np.empty_like(b)
    out[plan.order] = b
    return tuple(out[:, c] for c in range(k))


def route_batch(decide: Callable, keys, permits, ts_us, directory, group=None, owner_map=None):
    """Decide a batch whose requests arrived at this rank but may belong to any rank.

    ``decide(local_ids, permits, ts) -> (col0, col1[, ...])`` runs this rank's engine on
    the requests it owns (e.g. granted and remaining; a queueing engine adds the request
    ids it assigns, which a later ``route_cancel`` needs).  Returns the columns for this
    rank's own requests in their arrival order: granted/status as u8, remaining as i32,
    further columns as i64 (host path) or the int64 device tensors (device path)."""
    (lk, lp, lt), plan = route_requests(keys, permits, ts_us, directory, group, owner_map)
    cols = decide(lk, lp, lt)
    out = route_replies(plan, cols, group)
    if _is_cuda(out[0]):
        import torch
        return (out[0].to(torch.uint8), out[1].to(torch.int32)) + tuple(out[2:])
    return (out[0].astype(np.uint8), out[1].astype(np.int32)) + tuple(out[2:])


def route_cancel(cancel: Callable, keys, request_ids, directory, group=None, owner_map=None):
    """Cancel queued requests (CancelQueueState.TrySetCanceled, Q:480-506 / A:531-557)
    that may be queued on any rank: ``keys`` are global keys, ``request_ids`` the ids
    their owners assigned (``route_batch``'s extra reply column).  ``cancel(local_ids,
    request_ids) -> u8`` runs on the owner; a key unknown to the owner's directory has
    nothing queued.  Returns the hits in this rank's order.  Per owner, the cancels apply
    by source rank, then call order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if _is_cuda(keys):
        return _route_cancel_device(cancel, keys, request_ids, directory, world, group, owner_map)
    if isinstance(directory, DeviceDirectory):
        raise TypeError("route_cancel with a DeviceDirectory takes CUDA tensors of keys and request ids")
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.shape[0]
    owner = key_owner(keys, world, owner_map)
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    sc = torch.from_numpy(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = rc.numpy()
    payload = np.stack([keys[order].view(np.int64), np.asarray(request_ids, dtype=np.int64)[order]], axis=1)
    recv = torch.empty((int(recv_counts.sum()), 2), dtype=torch.int64)
    dist.all_to_all_single(recv, torch.from_numpy(np.ascontiguousarray(payload)),
                           output_split_sizes=recv_counts.tolist(), input_split_sizes=send_counts.tolist(),
                           group=group)
    r = recv.numpy()
    hit = np.zeros(r.shape[0], dtype=np.int64)
    if r.shape[0]:
        local = directory.lookup(r[:, 0].view(np.uint64))
        known = local != NO_ID
        if known.any():
            hit[known] = np.asarray(cancel(local[known], r[known, 1]), dtype=np.int64)
    back = torch.empty(n, dtype=torch.int64)
    dist.all_to_all_single(back, torch.from_numpy(hit), output_split_sizes=send_counts.tolist(),
                           input_split_sizes=recv_counts.tolist(), group=group)
    out = np.empty(n, dtype=np.uint8)
    out[order] = back.numpy()
    return out


def _route_cancel_device(cancel, keys, request_ids, directory, world, group, owner_map=None):
    """route_cancel's device path: (key, request id) pairs go to the owners through the
    route kernels (the id rides in the record's i64 payload), the owner's DeviceDirectory
    looks the keys up (a key it never assigned has nothing queued), ``cancel(local ids,
    request ids)`` gets the known pairs as int64 device tensors, and the hits come back
    through the reverse all-to-all.  Returns u8 hits (device tensor) in this rank's order."""
    import torch
    from . import _capi
    if not isinstance(directory, DeviceDirectory):
        raise TypeError("route_cancel with CUDA tensors needs a DeviceDirectory")
    keys, request_ids = _device_columns(keys, (request_ids, torch.int64))
    dev = keys.device
    zero = torch.zeros(keys.numel(), dtype=torch.int32, device=dev)
    pos, sc_l, rc_l, recv = _route_device(keys, zero, request_ids, world, group, owner_map)
    hit = torch.zeros(recv.shape[0], dtype=torch.int64, device=dev)
    if recv.shape[0]:
        local = directory.lookup(recv[:, 0])
        known = torch.nonzero(local != -1).flatten()
        if known.numel():
            h = cancel(local[known], recv[known, 1].contiguous())
            hit[known] = torch.as_tensor(np.asarray(h) if not _is_cuda(h) else h, device=dev).to(torch.int64)
    back = torch.empty((keys.numel(), 1), dtype=torch.int64, device=dev)
    _all_to_all(back, hit.view(-1, 1), sc_l, rc_l, group=group)
    out = torch.empty_like(back)
    lib = _capi.load()
    _check(lib.tbe_route_gather_device(pos.data_ptr(), keys.numel(), back.data_ptr(), 1, out.data_ptr(),
                                       device_stream(dev)))
    return out[:, 0].to(torch.uint8)


def device_stream(dev) -> int:
    """The current torch stream's handle for the device path.  The engine reads a NULL
    handle as "inputs complete at the call" (include/tbe.h), which the default stream's
    queued work is not, so the device path refuses it: run it inside
    torch.cuda.stream(torch.cuda.Stream(...))."""
    import torch
    h = torch.cuda.current_stream(dev).cuda_stream
    if not h:
        raise ValueError("cluster device path: set a non-default torch.cuda.Stream as current "
                         "(the default stream's NULL handle cannot order the engine's work)")
    return h


def _check(st: int) -> None:
    from . import _capi
    if st != _capi.TBE_OK:
        raise _capi.TbeError(st, "routing kernel launch failed")


# ------------------------------------------------------------------ approximate global tier
def approx_epoch(engine, counts, ts_us: int, stagger_us: int, mode: str = "clients",
                 group=None):
    """One refresh epoch of the ApproximateTokenBucket across ranks.

    ``engine`` exposes ``collect(counts)`` (A:430-435) and
    ``sync(all_counts, n_clients, my_client, ts_us, stagger_us)`` (A:439-508);
    ``counts`` is an int32 tensor [n_keys] on the engine's device.  Returns the drain
    log of this rank's queues."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    engine.collect(counts)
    if world == 1:
        return engine.sync(counts, 1, 0, ts_us, stagger_us, **_after_collective(counts))
    if mode == "clients":       # every rank is a client: exact prefix semantics
        allc = torch.empty(world * counts.numel(), dtype=counts.dtype, device=counts.device)
        _all_gather(allc, counts, group=group)
        return engine.sync(allc, world, rank, ts_us, stagger_us, **_after_collective(counts))
    if mode == "node":          # the node is one client: sum of the ranks' counts
        _all_reduce_sum(counts, group=group)
        return engine.sync(counts, 1, 0, ts_us, stagger_us, **_after_collective(counts))
    raise ValueError(f"unknown mode {mode!r}")


def _after_collective(t) -> dict:
    """The engine's sync replay reads the exchanged counts on its own stream: order it after
    the collective on the current stream (tbe_approx_sync_stream: an event, no host wait)."""
    if not _is_cuda(t):
        return {}
    import torch
    cur = torch.cuda.current_stream(t.device)
    if not cur.cuda_stream:     # the legacy default stream: no handle to order after
        cur.synchronize()
        return {}
    return {"stream": cur.cuda_stream}
