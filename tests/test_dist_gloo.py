"""World-size-2 tests of the multi-GPU protocol (cluster.py) with gloo on CPU.

* request routing: two ranks each receive requests for ANY key; after the all-to-all
  every key is decided by its owner.  Expected = one serial table processing, per step,
  rank 0's batch then rank 1's (the per-key serial order route_batch promises).
* approximate epochs: each rank is one client of the shared global tier; the counts are
  all-gathered and every rank replays the sync calls in client order.  Expected = the
  single-process multi-client reference (oracle.semantics.approx_refresh_all).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import _dist_workers as W

WORLD = 2


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, *args, world: int = WORLD):
    mp.start_processes(fn, args=(world, _port()) + args, nprocs=world, join=True,
                       start_method="spawn")


def test_key_owner_and_directory():
    """owner = top bits of mix64 for a power-of-two world, balanced; the
    host directory assigns a bijection of [0, capacity) in first-seen order."""
    from distributedratelimiting.redis_amd import cluster
    keys = np.arange(200_000, dtype=np.uint64)
    for world in (2, 4, 8):
        own = cluster.key_owner(keys, world)
        top = (cluster._mix64(keys) >> np.uint64(64 - (world.bit_length() - 1))).astype(np.int64)
        assert np.array_equal(own, top)
        cnt = np.bincount(own, minlength=world)
        assert cnt.min() > 0.97 * keys.size / world
    d = cluster.HostDirectory(1000)
    a = d.assign(np.array([7, 3, 7, 9], np.uint64))
    b = d.assign(np.array([9, 11, 3], np.uint64))
    assert a[0] == a[2] and len({int(a[0]), int(a[1]), int(a[3]), int(b[1])}) == 4
    assert b[0] == a[3] and b[2] == a[1]
    assert np.array_equal(cluster.scramble_walk(np.arange(4, dtype=np.uint64), 1000), np.array(
        [a[0], a[1], a[3], b[1]], np.uint64))                    # counters 0..3 in first-seen order
    ids = cluster.scramble_walk(np.arange(1000, dtype=np.uint64), 1000)
    assert np.array_equal(np.sort(ids), np.arange(1000, dtype=np.uint64))   # a bijection
    small = cluster.HostDirectory(2)
    out = small.assign(np.array([5, 6, 7], np.uint64))
    assert small.overflow and out[2] == cluster.NO_ID


@pytest.mark.parametrize("map_kind", ["hash", "balanced"])
def test_route_batch_matches_serial_reference(oracle_lib, tmp_path, map_kind):
    _spawn(W.tb_route_worker, str(tmp_path), map_kind)
    check_tb_route([np.load(tmp_path / f"tb_{r}.npz") for r in range(WORLD)])


def test_owner_map_validation():
    """a map that is not 4096 u8 owners below the world size is refused before
    any kernel reads it (route_requests / route_batch / route_cancel call key_owner or
    _device_map first)."""
    from distributedratelimiting.redis_amd import cluster
    keys = np.arange(1000, dtype=np.uint64)
    good = cluster.hash_owner_map(4)
    assert np.array_equal(cluster.key_owner(keys, 4, good), cluster.key_owner(keys, 4))
    for bad in (good[:100], np.concatenate([good, good]), np.full(4096, 4, np.uint8),
                np.full(4096, -1, np.int64), np.full(4096, 300, np.int64)):
        with pytest.raises(ValueError):
            cluster.key_owner(keys, 4, bad)
        with pytest.raises(ValueError):
            cluster._device_map(bad, None, 4)
    assert cluster._device_map(None, None, 4) is None


def test_owner_maps():
    """Table-driven ownership (include/tbe_cluster.h owner maps): the hash map reproduces
    the hash partition; the balanced map evens out a Zipf stream's owner loads that the
    hash partition leaves ~1.7x uneven (SURVEY.md §7 hard part iii), keeps the owners'
    shares of the key space level, is deterministic, and the host vnode function equals
    the engine's (tbe_key_vnode)."""
    from distributedratelimiting.redis_amd import _capi, cluster
    keys = np.arange(300_000, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    for world in (1, 2, 4, 8, 64):
        assert np.array_equal(cluster.key_owner(keys, world),
                              cluster.key_owner(keys, world, cluster.hash_owner_map(world)))
    lib = _capi.load()
    assert [lib.tbe_key_vnode(int(k)) for k in keys[:2000]] == cluster.key_vnode(keys[:2000]).tolist()
    # Zipf(1.1)-like loads: one key ~10% of the stream
    rng = np.random.default_rng(3)
    ranks = np.minimum(rng.zipf(1.1, 2_000_000), 10**9).astype(np.uint64)
    zkeys = cluster._mix64(ranks)                  # rank -> key
    loads = np.bincount(cluster.key_vnode(zkeys), minlength=cluster.OWNER_MAP_SIZE)
    for world in (4, 8):
        per_hash = np.bincount(cluster.key_owner(zkeys, world), minlength=world)
        m = cluster.balanced_owner_map(loads, world)
        assert np.array_equal(m, cluster.balanced_owner_map(loads.copy(), world))
        per_bal = np.bincount(cluster.key_owner(zkeys, world, m), minlength=world)
        assert per_hash.max() / per_hash.mean() > 1.3
        assert per_bal.max() / per_bal.mean() < 1.01
        nv = np.bincount(m, minlength=world)
        assert nv.sum() == cluster.OWNER_MAP_SIZE and nv.min() > 0
        cap = cluster.keys_per_rank(10**9, world, owner_map=m)
        assert cap >= 10**9 * nv.max() // cluster.OWNER_MAP_SIZE
    # no load at all: the shares of the key space stay level
    m = cluster.balanced_owner_map(np.zeros(cluster.OWNER_MAP_SIZE, np.int64), 8)
    assert np.bincount(m, minlength=8).tolist() == [512] * 8
    # config C at 8 GPUs (1e9 keys): the uncapped map gives the hot key's owner few virtual
    # nodes and every other owner more than 2^27 keys (a third pass, unpacked records, no
    # hot runs); with n_keys no table leaves the packed two-pass layout, and the load is
    # still more even than the hash partition's
    for world in (4, 8):
        per_hash = np.bincount(cluster.key_owner(zkeys, world), minlength=world)
        free = cluster.balanced_owner_map(loads, world)
        m = cluster.balanced_owner_map(loads, world, n_keys=10**9)
        cap_v = cluster.max_vnodes_per_owner(10**9, world)
        assert np.bincount(m, minlength=world).max() <= cap_v
        if world == 8:   # (at 4 GPUs the even share, 2.5e8 keys, is past the limit anyway)
            assert cluster.keys_per_rank(10**9, world, owner_map=m) <= cluster.PACKED_KEYS_MAX
            assert cluster.keys_per_rank(10**9, world, owner_map=free) > cluster.PACKED_KEYS_MAX
        per_bal = np.bincount(cluster.key_owner(zkeys, world, m), minlength=world)
        assert per_bal.max() / per_bal.mean() < per_hash.max() / per_hash.mean()
    # the cap never goes below the even share, and is the limit when the share is small
    assert cluster.max_vnodes_per_owner(10**9, 8) >= 512
    assert cluster.max_vnodes_per_owner(4 * 10**9, 8) == 512
    assert cluster.max_vnodes_per_owner(10**6, 8) == cluster.OWNER_MAP_SIZE


def check_tb_route(res):
    """Expected: one serial table; per step rank 0's batch, then rank 1's, ..."""
    WORLD = len(res)
    from oracle import cref
    from oracle.semantics import fill_rate_per_second
    rate = fill_rate_per_second(W.TB["tokens_per_period"], W.TB["period_ticks"])
    ref = cref.CTokenBucket(W.TB["n_keys"], W.TB["token_limit"], rate)
    for s in range(W.TB_STEPS):
        batches = [W.tb_batch(r, s) for r in range(WORLD)]
        k = np.concatenate([b[0] for b in batches])
        p = np.concatenate([b[1] for b in batches])
        t = np.concatenate([b[2] for b in batches])
        g, rem = ref.acquire_batch(k, p, t)
        for r in range(WORLD):
            sl = slice(r * W.TB_N, (r + 1) * W.TB_N)
            assert np.array_equal(res[r][f"g{s}"], g[sl]), (s, r)
            assert np.array_equal(res[r][f"r{s}"], rem[sl]), (s, r)
    from distributedratelimiting.redis_amd import cluster
    v, t = ref.export_state()
    seen = 0
    omap = res[0]["owner_map"] if "owner_map" in res[0] else None
    for r in range(WORLD):
        keys, ids = res[r]["dir_keys"].astype(np.int64), res[r]["dir_ids"].astype(np.int64)
        assert np.all(cluster.key_owner(keys.astype(np.uint64), WORLD, omap) == r)   # the owner's keys only
        assert np.array_equal(res[r]["t"][ids], t[keys])
        assert np.array_equal(res[r]["v"][ids].view(np.int64), v[keys].view(np.int64))
        seen += keys.size
    assert seen == np.unique(np.concatenate([W.tb_batch(r, s)[0] for r in range(WORLD)
                                             for s in range(W.TB_STEPS)])).size
    ref.close()


def test_approx_epoch_clients_matches_multi_client_reference(tmp_path):
    _spawn(W.ap_epoch_worker, str(tmp_path), "clients")
    check_approx([np.load(tmp_path / f"ap_clients_{r}.npz") for r in range(WORLD)], "clients")


def check_approx(res, mode):
    """Expected: the single-process multi-client reference.  clients: client r syncs at
    T + r*stagger and sees clients < r (approx_refresh_all); node: the ranks' counts
    summed into ONE sync call per key, whose reply every rank applies."""
    WORLD = len(res)
    from oracle.semantics import ApproxClient, ApproxGlobalTable, approx_refresh_all
    A = W.AP
    clients = [ApproxClient(A["token_limit"], A["tokens_per_period"], A["period_ticks"],
                            A["queue_limit"], A["order"]) for _ in range(WORLD)]
    for c in clients:
        for k in range(A["n_keys"]):
            c.st(k)
    table = ApproxGlobalTable(clients[0].decay_rate)
    statuses = [[] for _ in range(WORLD)]
    logs = [[] for _ in range(WORLD)]
    rids = [0] * WORLD
    for e in range(W.AP_EPOCHS):
        for r in range(WORLD):
            keys, permits = W.ap_batch(r, e)
            for k, p in zip(keys.tolist(), permits.tolist()):
                statuses[r].append(clients[r].wait(k, p, rids[r])[0])
                rids[r] += 1
        if mode == "clients":
            lg = approx_refresh_all(clients, table, W.ap_epoch_ts(e), W.AP_STAGGER, range(A["n_keys"]))
        else:
            counts = [c.collect() for c in clients]
            for k in range(A["n_keys"]):
                g, period, _ = table.sync(f"approx:{k}", sum(c.get(k, 0) for c in counts), W.ap_epoch_ts(e))
                for c in clients:
                    c.apply_sync(k, g, period)
            lg = [c.drain() for c in clients]
        for r in range(WORLD):
            logs[r].extend((e, k, i) for k, i in lg[r])
    for r in range(WORLD):
        assert res[r]["status"].tolist() == statuses[r]
        assert [tuple(x) for x in res[r]["log"].tolist()] == logs[r]
        exp = np.array([[s.local, s.global_, s.est, s.qcount]
                        for _, s in sorted(clients[r].keys.items())], dtype=np.float64)
        assert np.array_equal(res[r]["state"], exp)
    # the exchange did something: both clients see a non-trivial global score
    assert res[0]["state"][:, 1].max() > 0
    assert any(len(l) for l in logs)


def test_approx_epoch_node_mode_sums_counts(tmp_path):
    """mode="node": the ranks act as ONE client; every rank's sync sees the summed count."""
    _spawn(W.ap_epoch_worker, str(tmp_path), "node")
    res = [np.load(tmp_path / f"ap_node_{r}.npz") for r in range(WORLD)]
    # both ranks replay identical sync calls -> identical global scores and estimates
    assert np.array_equal(res[0]["state"][:, 1:3], res[1]["state"][:, 1:3])
    check_approx(res, "node")


# ---- world size 8: the protocol an 8-GPU node runs, rehearsed with
# eight gloo ranks on the CPU -- routing under the hash (§8e) and balanced owner maps, queued
# waits with routed cancels, and both approximate exchange modes -- against the same serial
# restatements.  Multi-GPU figures stay unmeasured on hardware; this checks the protocol.
W8 = 8


@pytest.mark.timeout(600)
@pytest.mark.parametrize("map_kind", ["hash", "balanced"])
def test_world8_route_batch_matches_serial_reference(oracle_lib, tmp_path, map_kind):
    _spawn(W.tb_route_worker, str(tmp_path), map_kind, world=W8)
    res = [np.load(tmp_path / f"tb_{r}.npz") for r in range(W8)]
    check_tb_route(res)
    assert all(res[r]["dir_keys"].size > 0 for r in range(W8))   # every owner received keys


@pytest.mark.timeout(600)
def test_world8_route_wait_and_cancel_matches_serial_reference(tmp_path):
    _spawn(W.q_route_worker, str(tmp_path), world=W8)
    check_q_route([np.load(tmp_path / f"q_{r}.npz") for r in range(W8)])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["clients", "node"])
def test_world8_approx_epoch_matches_reference(tmp_path, mode):
    _spawn(W.ap_epoch_worker, str(tmp_path), mode, world=W8)
    res = [np.load(tmp_path / f"ap_{mode}_{r}.npz") for r in range(W8)]
    if mode == "node":
        for r in range(1, W8):
            assert np.array_equal(res[0]["state"][:, 1:3], res[r]["state"][:, 1:3])
    check_approx(res, mode)


def test_route_wait_and_cancel_matches_serial_reference(tmp_path):
    """Queued waits routed to their owners, then cancels of some of them routed the same
    way (cluster.route_cancel), then a replenish tick on every rank.  Expected = one
    serial queueing table: per step rank 0's batch, rank 1's, the cancels, the tick."""
    _spawn(W.q_route_worker, str(tmp_path))
    check_q_route([np.load(tmp_path / f"q_{r}.npz") for r in range(WORLD)])


def check_q_route(res):
    WORLD = len(res)
    from oracle.semantics import QueueingTokenBucketTable, TokenBucketConfig
    from distributedratelimiting.redis_amd import cluster
    Q = W.Q
    ref = QueueingTokenBucketTable(TokenBucketConfig.from_options(
        Q["token_limit"], Q["tokens_per_period"], Q["period_ticks"]), Q["queue_limit"], Q["order"])
    ref_id = lambda s, src, i: (s * WORLD + src) * W.Q_N + i   # noqa: E731
    owner_id = {}   # (owner rank, owner-assigned id) -> reference id
    total_hits = 0
    for s in range(W.Q_STEPS):
        batches = [W.q_batch(r, s) for r in range(WORLD)]
        for src, (k, p, t) in enumerate(batches):
            exp = [ref.acquire(int(k[i]), int(p[i]), int(t[i]), ref_id(s, src, i)) for i in range(W.Q_N)]
            assert res[src][f"st{s}"].tolist() == [e[0] for e in exp], (s, src)
            assert res[src][f"rem{s}"].tolist() == [e[1] for e in exp], (s, src)
            own = cluster.key_owner(k, WORLD)
            for i, x in enumerate(res[src][f"ids{s}"].tolist()):
                owner_id[(int(own[i]), x)] = ref_id(s, src, i)
        for src, (k, _, _) in enumerate(batches):
            pick = W.q_cancel_pick(res[src][f"st{s}"])
            want = [int(ref.cancel(int(k[i]), ref_id(s, src, int(i)))) for i in pick]
            assert res[src][f"hit{s}"].tolist() == want, (s, src)
            total_hits += sum(want)
        exp_log = ref.refresh(W.q_refresh_ts(s))
        got = []
        for r in range(WORLD):
            gkey = dict(zip(res[r]["dir_ids"].tolist(), res[r]["dir_keys"].tolist()))
            for lk, x, rem in res[r][f"log{s}"].tolist():
                got.append((gkey[lk], owner_id[(r, x)], rem))
        got.sort(key=lambda e: e[0])   # stable: per-key drain order kept
        assert got == exp_log, s
    assert total_hits > 0
