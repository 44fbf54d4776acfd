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


def _spawn(fn, *args):
    mp.start_processes(fn, args=(WORLD, _port()) + args, nprocs=WORLD, join=True,
                       start_method="spawn")


def test_shard_batch_partition():
    from distributedratelimiting.redis_amd import cluster
    keys = np.array([5, 2, 7, 4, 9, 0, 3], dtype=np.uint64)
    parts = cluster.shard_batch(keys, np.arange(7), np.arange(7) * 10, 3)
    seen = np.concatenate([p[0] for p in parts])
    assert sorted(seen.tolist()) == list(range(7))
    for r, (idx, lk, pp, tt) in enumerate(parts):
        assert np.all(keys[idx] % 3 == r)
        assert np.all(np.diff(idx) > 0)                      # arrival order kept
        assert np.array_equal(lk * 3 + r, keys[idx])
        assert np.array_equal(pp, idx) and np.array_equal(tt, idx * 10)


def test_route_batch_matches_serial_reference(oracle_lib, tmp_path):
    from oracle import cref
    from oracle.semantics import fill_rate_per_second
    _spawn(W.tb_route_worker, str(tmp_path))
    res = [np.load(tmp_path / f"tb_{r}.npz") for r in range(WORLD)]

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
    v, t = ref.export_state()
    for r in range(WORLD):
        keys = np.arange(r, W.TB["n_keys"], WORLD)
        n = keys.size
        assert np.array_equal(res[r]["t"][:n], t[keys])
        assert np.array_equal(res[r]["v"][:n].view(np.int64), v[keys].view(np.int64))
    ref.close()


def test_approx_epoch_clients_matches_multi_client_reference(tmp_path):
    from oracle.semantics import ApproxClient, ApproxGlobalTable, approx_refresh_all
    _spawn(W.ap_epoch_worker, str(tmp_path), "clients")
    res = [np.load(tmp_path / f"ap_clients_{r}.npz") for r in range(WORLD)]

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
        lg = approx_refresh_all(clients, table, W.ap_epoch_ts(e), W.AP_STAGGER, range(A["n_keys"]))
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
    assert res[0]["state"][:, 1].max() > 0
