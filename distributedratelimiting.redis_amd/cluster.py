"""Multi-GPU layer: one engine per GPU (one process per rank), keys hash-partitioned.

The reference distributes by letting many client processes share one Redis key space
(SURVEY.md §2).  Here every key has exactly one owner GPU holding its bucket state, so
the token-bucket paths need no collective at all when ingest is already partitioned
(the benchmark mode).  Two exchanges exist:

* ``route_batch``: when requests arrive at arbitrary ranks, one all-to-all sends each to
  its owner (ordered by source rank, then arrival index) and a reverse all-to-all
  returns the replies.  The combined order is a valid serial order of the reference:
  per key, rank 0's requests of this step precede rank 1's, and so on.
* ``route_cancel``: cancellations of queued requests travel to the key's owner the
  same way (one all-to-all of (key, request id), one of the hits back).
* ``approx_epoch``: the ApproximateTokenBucket global tier.  Each rank is one client
  (A:9-599) holding a local tier for every shared key; at every refresh epoch the
  per-key consumed counts are exchanged -- all-gather for exact per-client prefix
  semantics (client r's sync call sees clients 0..r-1, SURVEY.md §8e option 2), or
  all-reduce when the node acts as ONE client (option 1) -- and every rank replays
  the same sync calls on its replica of the global tier.

With backend "nccl" (RCCL on ROCm) the collectives run over xGMI on device tensors;
tests drive the same code with "gloo" on CPU tensors.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


# ------------------------------------------------------------------ key partitioning
def key_owner(keys: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of each (dense) key id.  Ids are assumed scrambled by the caller's
    string-key directory (PTB:42 builds ``InstanceName + resourceID``); with dense
    uniform ids ``key % world`` balances exactly."""
    return (np.asarray(keys, dtype=np.uint64) % np.uint64(world)).astype(np.int64)


def local_key(keys: np.ndarray, world: int) -> np.ndarray:
    """Dense id of a key inside its owner's table: ``key // world``."""
    return np.asarray(keys, dtype=np.uint64) // np.uint64(world)


def keys_per_rank(n_keys: int, world: int) -> int:
    return (n_keys + world - 1) // world


def shard_batch(keys, permits, ts_us, world: int):
    """Stable split of one batch by owner: for each rank r, (arrival indices, local keys,
    permits, ts).  Arrival order is preserved inside every shard."""
    keys = np.asarray(keys, dtype=np.uint64)
    owner = key_owner(keys, world)
    order = np.argsort(owner, kind="stable")
    bounds = np.searchsorted(owner[order], np.arange(world + 1))
    out = []
    for r in range(world):
        idx = order[bounds[r]:bounds[r + 1]]
        out.append((idx, local_key(keys[idx], world), np.asarray(permits)[idx],
                    np.asarray(ts_us)[idx]))
    return out


# ------------------------------------------------------------------ all-to-all routing
def route_batch(decide: Callable, keys, permits, ts_us, group=None, device=None):
    """Decide a batch whose requests arrived at this rank but may belong to any rank.

    ``decide(local_keys, permits, ts) -> (granted u8, remaining i32[, extra...])`` runs
    this rank's engine on the requests it owns.  Returns (granted, remaining) for this
    rank's own requests in their arrival order, plus any extra int64 reply column
    ``decide`` returns (a queueing engine's request ids, which the owner assigns and a
    later ``route_cancel`` needs).  Two all-to-alls (requests out, replies back)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.shape[0]
    owner = key_owner(keys, world)
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    to = (lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)) if device else \
        (lambda a: torch.from_numpy(np.ascontiguousarray(a)))
    sc = to(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = rc.cpu().numpy()
    # one int64 record per field keeps the exchange to three all-to-alls of one dtype
    payload = np.stack([local_key(keys[order], world).astype(np.int64),
                        np.asarray(permits, dtype=np.int64)[order],
                        np.asarray(ts_us, dtype=np.int64)[order]], axis=1)
    recv = torch.empty((int(recv_counts.sum()), 3), dtype=torch.int64, device=device)
    dist.all_to_all_single(recv, to(payload), output_split_sizes=recv_counts.tolist(),
                           input_split_sizes=send_counts.tolist(), group=group)
    r = recv.cpu().numpy()
    outs = decide(r[:, 0].astype(np.uint64), r[:, 1].astype(np.int32), r[:, 2])
    cols = len(outs)
    reply = np.stack([np.asarray(x, dtype=np.int64).reshape(-1) for x in outs], axis=1) \
        if r.shape[0] else np.zeros((0, cols), dtype=np.int64)
    back = torch.empty((n, cols), dtype=torch.int64, device=device)
    dist.all_to_all_single(back, to(reply), output_split_sizes=send_counts.tolist(),
                           input_split_sizes=recv_counts.tolist(), group=group)
    b = back.cpu().numpy()
    res = [np.empty(n, dtype=dt) for dt in [np.uint8, np.int32] + [np.int64] * (cols - 2)]
    for c in range(cols):
        res[c][order] = b[:, c]
    return tuple(res)


def route_cancel(cancel: Callable, keys, request_ids, group=None, device=None):
    """Cancel queued requests (CancelQueueState.TrySetCanceled, Q:480-506 / A:531-557)
    that may be queued on any rank: ``keys`` are global key ids, ``request_ids`` the ids
    their owners assigned (``route_batch``'s extra reply column).  ``cancel(local_keys,
    request_ids) -> u8`` runs on the owner (``QueueingTokenBucketEngine.cancel``).
    Returns the u8 hits in this rank's order.  Per owner, the cancels apply by source
    rank, then call order.  Two all-to-alls."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.shape[0]
    owner = key_owner(keys, world)
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    to = (lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)) if device else \
        (lambda a: torch.from_numpy(np.ascontiguousarray(a)))
    sc = to(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = rc.cpu().numpy()
    payload = np.stack([local_key(keys[order], world).astype(np.int64),
                        np.asarray(request_ids, dtype=np.int64)[order]], axis=1)
    recv = torch.empty((int(recv_counts.sum()), 2), dtype=torch.int64, device=device)
    dist.all_to_all_single(recv, to(payload), output_split_sizes=recv_counts.tolist(),
                           input_split_sizes=send_counts.tolist(), group=group)
    r = recv.cpu().numpy()
    hit = np.asarray(cancel(r[:, 0].astype(np.uint64), r[:, 1]), dtype=np.int64) if r.shape[0] \
        else np.zeros(0, dtype=np.int64)
    back = torch.empty(n, dtype=torch.int64, device=device)
    dist.all_to_all_single(back, to(hit), output_split_sizes=send_counts.tolist(),
                           input_split_sizes=recv_counts.tolist(), group=group)
    out = np.empty(n, dtype=np.uint8)
    out[order] = back.cpu().numpy()
    return out


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
        return engine.sync(counts, 1, 0, ts_us, stagger_us)
    if mode == "clients":       # every rank is a client: exact prefix semantics
        allc = torch.empty(world * counts.numel(), dtype=counts.dtype, device=counts.device)
        dist.all_gather_into_tensor(allc, counts, group=group)
        return engine.sync(allc, world, rank, ts_us, stagger_us)
    if mode == "node":          # the node is one client: sum of the ranks' counts
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        return engine.sync(counts, 1, 0, ts_us, stagger_us)
    raise ValueError(f"unknown mode {mode!r}")
