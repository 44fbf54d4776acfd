"""Rank bodies for tests/test_dist_gloo.py (world_size 2, gloo on CPU).

The engines here are the oracle stand-ins (tests may use oracle/): the point is the
cluster protocol of distributedratelimiting.redis_amd/cluster.py -- routing and the
approximate-limiter epoch -- which is the same code that drives the HIP engines over
RCCL on a GPU node.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _init(rank: int, world: int, port: int):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


# ------------------------------------------------------------------ token bucket routing
TB = dict(n_keys=1000, token_limit=5, tokens_per_period=1, period_ticks=10_000_000)
TB_STEPS, TB_N = 4, 3000


def tb_batch(rank: int, step: int):
    rng = np.random.default_rng(1000 * rank + step)
    keys = rng.integers(0, TB["n_keys"], TB_N, dtype=np.uint64)
    permits = rng.integers(0, 4, TB_N, dtype=np.int32)
    ts = 1_760_000_000_000_000 + step * 700_000 + np.sort(rng.integers(0, 700_000, TB_N))
    return keys, permits, ts.astype(np.int64)


def tb_owner_map(world: int, kind: str):
    """None (hash partition) or the balanced owner map of the test's whole stream (every
    rank computes the same one from the same loads)."""
    from distributedratelimiting.redis_amd import cluster
    if kind != "balanced":
        return None
    keys = np.concatenate([tb_batch(r, s)[0] for r in range(world) for s in range(TB_STEPS)])
    return cluster.balanced_owner_map(np.bincount(cluster.key_vnode(keys), minlength=cluster.OWNER_MAP_SIZE), world)


def tb_route_worker(rank: int, world: int, port: int, out_dir: str, map_kind: str = "hash"):
    dist = _init(rank, world, port)
    from oracle import cref
    from oracle.semantics import fill_rate_per_second
    from distributedratelimiting.redis_amd import cluster

    rate = fill_rate_per_second(TB["tokens_per_period"], TB["period_ticks"])
    omap = tb_owner_map(world, map_kind)
    cap = cluster.keys_per_rank(TB["n_keys"], world, owner_map=omap)
    directory = cluster.HostDirectory(cap)
    ref = cref.CTokenBucket(cap, TB["token_limit"], rate)
    out = {} if omap is None else {"owner_map": omap}
    for s in range(TB_STEPS):
        k, p, t = tb_batch(rank, s)
        g, r = cluster.route_batch(lambda lk, lp, lt: ref.acquire_batch(lk, lp, lt), k, p, t, directory,
                                   owner_map=omap)
        out[f"g{s}"], out[f"r{s}"] = g, r
    v, tt = ref.export_state()
    out["v"], out["t"] = v, tt
    out["dir_keys"] = np.array(list(directory.ids.keys()), dtype=np.uint64)
    out["dir_ids"] = np.array(list(directory.ids.values()), dtype=np.uint64)
    np.savez(os.path.join(out_dir, f"tb_{rank}.npz"), **out)
    ref.close()
    dist.barrier()
    dist.destroy_process_group()


# ------------------------------------------------------------------ approximate epochs
AP = dict(n_keys=24, token_limit=8, tokens_per_period=4, period_ticks=10_000_000,
          queue_limit=6, order=0)
AP_EPOCHS, AP_N, AP_STAGGER = 5, 60, 1500


def ap_batch(rank: int, epoch: int):
    rng = np.random.default_rng(77 + 31 * rank + 1009 * epoch)
    keys = rng.integers(0, AP["n_keys"], AP_N)
    permits = rng.integers(0, 5, AP_N)
    return keys, permits


def ap_epoch_ts(epoch: int) -> int:
    return 1_760_000_000_000_000 + (epoch + 1) * 1_000_000 + epoch * 37_000


class OracleApproxEngine:
    """Stand-in with the ApproximateEngine collect/sync contract: this rank's client plus a
    replica of the global tier that every rank updates with the same sync calls."""

    def __init__(self):
        from oracle.semantics import ApproxClient, ApproxGlobalTable
        self.client = ApproxClient(AP["token_limit"], AP["tokens_per_period"], AP["period_ticks"],
                                   AP["queue_limit"], AP["order"])
        for k in range(AP["n_keys"]):
            self.client.st(k)
        self.table = ApproxGlobalTable(self.client.decay_rate)

    def collect(self, counts):
        c = self.client.collect()
        for k in range(AP["n_keys"]):
            counts[k] = c.get(k, 0)

    def sync(self, all_counts, n_clients, my_client, ts_us, stagger_us):
        K = AP["n_keys"]
        a = all_counts.numpy()
        for r in range(n_clients):
            for k in range(K):
                g, period, _ = self.table.sync(f"approx:{k}", int(a[r * K + k]), ts_us + r * stagger_us)
                if r == my_client:
                    self.client.apply_sync(k, g, period)
        return self.client.drain()


def ap_epoch_worker(rank: int, world: int, port: int, out_dir: str, mode: str):
    import torch
    dist = _init(rank, world, port)
    from distributedratelimiting.redis_amd import cluster

    eng = OracleApproxEngine()
    statuses, logs = [], []
    rid = 0
    for e in range(AP_EPOCHS):
        keys, permits = ap_batch(rank, e)
        for k, p in zip(keys.tolist(), permits.tolist()):
            st, _ = eng.client.wait(k, p, rid)
            statuses.append(st)
            rid += 1
        counts = torch.zeros(AP["n_keys"], dtype=torch.int32)
        logs.append(cluster.approx_epoch(eng, counts, ap_epoch_ts(e), AP_STAGGER, mode=mode))
    state = np.array([[s.local, s.global_, s.est, s.qcount]
                      for _, s in sorted(eng.client.keys.items())], dtype=np.float64)
    np.savez(os.path.join(out_dir, f"ap_{mode}_{rank}.npz"), status=np.array(statuses),
             log=np.array([(e, k, r) for e, lg in enumerate(logs) for k, r in lg],
                          dtype=np.int64).reshape(-1, 3),
             state=state)
    dist.barrier()
    dist.destroy_process_group()


# ------------------------------------------------------------------ queued waits + cancels
Q = dict(n_keys=40, token_limit=4, tokens_per_period=1, period_ticks=10_000_000, queue_limit=5, order=0)
Q_STEPS, Q_N, Q_T0 = 3, 300, 1_760_000_000_000_000


def q_batch(rank: int, step: int):
    rng = np.random.default_rng(555 + 100 * rank + step)
    keys = rng.integers(0, Q["n_keys"], Q_N, dtype=np.uint64)
    permits = rng.choice([0, 1, 1, 2, 3], Q_N).astype(np.int32)
    ts = Q_T0 + step * 700_000 + np.sort(rng.integers(0, 1_000, Q_N))
    return keys, permits, ts.astype(np.int64)


def q_cancel_pick(status) -> np.ndarray:
    """A third of the queued requests, plus a few that are not queued."""
    return np.array([i for i in range(Q_N) if (i % 3 == 0 and status[i] == 2) or i % 17 == 5],
                    dtype=np.int64)


def q_refresh_ts(step: int) -> int:
    return Q_T0 + step * 700_000 + 500_000


def q_route_worker(rank: int, world: int, port: int, out_dir: str):
    dist = _init(rank, world, port)
    from oracle.semantics import QueueingTokenBucketTable, TokenBucketConfig
    from distributedratelimiting.redis_amd import cluster

    tab = QueueingTokenBucketTable(TokenBucketConfig.from_options(
        Q["token_limit"], Q["tokens_per_period"], Q["period_ticks"]), Q["queue_limit"], Q["order"])
    next_id = [0]

    def wait(lk, lp, lt):   # the owner's engine: WaitAsync, ids assigned in arrival order
        st, rem, ids = [], [], []
        for k, p, t in zip(lk.tolist(), lp.tolist(), lt.tolist()):
            s, r, _ = tab.acquire(k, p, t, next_id[0])
            st.append(s)
            rem.append(r)
            ids.append(next_id[0])
            next_id[0] += 1
        return np.array(st), np.array(rem), np.array(ids)

    def cancel(lk, ids):
        return np.array([int(tab.cancel(int(k), int(i))) for k, i in zip(lk.tolist(), ids.tolist())])

    directory = cluster.HostDirectory(Q["n_keys"])
    out = {}
    for s in range(Q_STEPS):
        k, p, t = q_batch(rank, s)
        st, rem, ids = cluster.route_batch(wait, k, p, t, directory)
        pick = q_cancel_pick(st)
        hit = cluster.route_cancel(cancel, k[pick], ids[pick], directory)
        log = tab.refresh(q_refresh_ts(s))
        out[f"st{s}"], out[f"rem{s}"], out[f"ids{s}"], out[f"hit{s}"] = st, rem, ids, hit
        out[f"log{s}"] = np.array(log, dtype=np.int64).reshape(-1, 3)
    out["dir_keys"] = np.array(list(directory.ids.keys()), dtype=np.uint64)
    out["dir_ids"] = np.array(list(directory.ids.values()), dtype=np.uint64)
    np.savez(os.path.join(out_dir, f"q_{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


# ------------------------------------------------------------------ HIP engines (GPU tests)
# The same three protocols with this rank's decisions made by the HIP engine (libtbe.so)
# on cuda:0: the GPU test starts two such ranks on the one GPU of its box, over gloo (RCCL
# refuses two ranks on one device).  path "host": numpy batches, HostDirectory, the
# engine's host-buffer calls; path "device": CUDA tensors end to end -- route kernels,
# DeviceDirectory, device-buffer engine calls -- with gloo's collectives staged through
# host memory by cluster.py.
def _hip_setup():
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)     # the device path refuses the NULL stream
    torch.cuda.set_stream(stream)
    return torch, dev, stream


def _owned_keys(batch_fn, steps: int, rank: int, world: int, owner_map=None) -> np.ndarray:
    """Every key this rank owns among all ranks' batches (each rank can compute them)."""
    from distributedratelimiting.redis_amd import cluster
    keys = np.unique(np.concatenate([batch_fn(r, s)[0] for r in range(world) for s in range(steps)]))
    return keys[cluster.key_owner(keys, world, owner_map) == rank].astype(np.uint64)


def _dir_ids(directory, keys: np.ndarray, torch, dev) -> np.ndarray:
    from distributedratelimiting.redis_amd import cluster
    if isinstance(directory, cluster.DeviceDirectory):
        return directory.lookup(torch.from_numpy(keys.view(np.int64)).to(dev)).cpu().numpy().view(np.uint64)
    return directory.lookup(keys)


def tb_route_worker_hip(rank: int, world: int, port: int, out_dir: str, path: str, map_kind: str = "hash"):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import TokenBucketEngine, cluster

    omap = tb_owner_map(world, map_kind)
    cap = cluster.keys_per_rank(TB["n_keys"], world, owner_map=omap)
    eng = TokenBucketEngine(cap, TB["token_limit"], TB["tokens_per_period"], TB["period_ticks"], device=0)
    out = {} if omap is None else {"owner_map": omap}
    if path == "device":
        directory = cluster.DeviceDirectory(cap, device=0)

        def decide(lk, lp, lt):
            g = torch.empty(lk.numel(), dtype=torch.uint8, device=dev)
            r = torch.empty(lk.numel(), dtype=torch.int32, device=dev)
            eng.acquire_batch_device(lk, lp, lt, g, r, stream=stream.cuda_stream)
            return g, r
        for s in range(TB_STEPS):
            k, p, t = (torch.from_numpy(np.asarray(x).view(np.int64) if x.dtype == np.uint64 else x).to(dev)
                       for x in tb_batch(rank, s))
            g, r = cluster.route_batch(decide, k, p, t, directory, owner_map=omap)
            out[f"g{s}"], out[f"r{s}"] = g.cpu().numpy(), r.cpu().numpy()
    else:
        directory = cluster.HostDirectory(cap)
        for s in range(TB_STEPS):
            k, p, t = tb_batch(rank, s)
            g, r = cluster.route_batch(lambda lk, lp, lt: eng.acquire_batch(lk, lp, lt), k, p, t, directory,
                                       owner_map=omap)
            out[f"g{s}"], out[f"r{s}"] = g, r
    eng.synchronize()
    v, tt = eng.export_state()
    out["v"], out["t"] = v, tt
    owned = _owned_keys(tb_batch, TB_STEPS, rank, world, omap)
    out["dir_keys"], out["dir_ids"] = owned, _dir_ids(directory, owned, torch, dev)
    np.savez(os.path.join(out_dir, f"tb_{rank}.npz"), **out)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def q_route_worker_hip(rank: int, world: int, port: int, out_dir: str, path: str):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, cluster

    eng = QueueingTokenBucketEngine(Q["n_keys"], Q["token_limit"], Q["tokens_per_period"], Q["period_ticks"],
                                    Q["queue_limit"], Q["order"], device=0)
    next_id = [0]
    device = path == "device"

    def wait(lk, lp, lt):   # the owner's engine: WaitAsync, ids assigned in arrival order
        m = lk.shape[0]
        base = next_id[0]
        next_id[0] += m
        if device:
            st = torch.empty(m, dtype=torch.uint8, device=dev)
            rem = torch.empty(m, dtype=torch.int32, device=dev)
            if m:
                eng.wait_batch_device(lk, lp, lt, st, rem, base, wait=True, stream=stream.cuda_stream)
            return st, rem, base + torch.arange(m, dtype=torch.int64, device=dev)
        st, rem, _ = eng.wait_batch(lk, lp, lt, base)
        return st, rem, base + np.arange(m, dtype=np.int64)

    def cancel(lk, ids):    # host-buffer cancel (tbe_queue_cancel); device inputs staged
        if device:
            eng.synchronize()
            return eng.cancel(lk.cpu().numpy().view(np.uint64), ids.cpu().numpy())
        return eng.cancel(lk, ids)

    directory = cluster.DeviceDirectory(Q["n_keys"], device=0) if device else cluster.HostDirectory(Q["n_keys"])
    out = {}
    for s in range(Q_STEPS):
        k, p, t = q_batch(rank, s)
        if device:
            kd, pd, td = (torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev) for x in (k, p, t))
            st, rem, ids = (x.cpu().numpy() for x in cluster.route_batch(wait, kd, pd, td, directory))
        else:
            st, rem, ids = cluster.route_batch(wait, k, p, t, directory)
        pick = q_cancel_pick(st)
        if device:
            hit = cluster.route_cancel(cancel, torch.from_numpy(k[pick].view(np.int64)).to(dev),
                                       torch.from_numpy(ids[pick].astype(np.int64)).to(dev), directory).cpu().numpy()
        else:
            hit = cluster.route_cancel(cancel, k[pick], ids[pick], directory)
        lk, li, lr = eng.refresh(q_refresh_ts(s))
        out[f"st{s}"], out[f"rem{s}"], out[f"ids{s}"], out[f"hit{s}"] = st, rem, ids, hit
        out[f"log{s}"] = np.stack([lk.astype(np.int64), li, lr.astype(np.int64)], axis=1).reshape(-1, 3)
    owned = _owned_keys(q_batch, Q_STEPS, rank, world)
    out["dir_keys"], out["dir_ids"] = owned, _dir_ids(directory, owned, torch, dev)
    np.savez(os.path.join(out_dir, f"q_{rank}.npz"), **out)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def ap_epoch_worker_hip(rank: int, world: int, port: int, out_dir: str, mode: str):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import ApproximateEngine, cluster

    eng = ApproximateEngine(AP["n_keys"], AP["token_limit"], AP["tokens_per_period"], AP["period_ticks"],
                            AP["queue_limit"], AP["order"], device=0)
    statuses, logs = [], []
    rid = 0
    for e in range(AP_EPOCHS):
        keys, permits = ap_batch(rank, e)
        st, _, _ = eng.acquire_batch(keys, permits, wait=True, id_base=rid)
        statuses.extend(st.tolist())
        rid += keys.shape[0]
        counts = torch.zeros(AP["n_keys"], dtype=torch.int32, device=dev)
        lk, li, _ = cluster.approx_epoch(eng, counts, ap_epoch_ts(e), AP_STAGGER, mode=mode)
        logs.append(list(zip(lk.tolist(), li.tolist())))
    # [local, global, est, queued permits (_queueCount)] per key, as the oracle client's
    state = np.array([[lo, gl, est, sum(p for _, p in eng.queue_of(k))] for k, (lo, gl, est, _, _) in
                      enumerate(eng.local_state(k) for k in range(AP["n_keys"]))], dtype=np.float64)
    np.savez(os.path.join(out_dir, f"ap_{mode}_{rank}.npz"), status=np.array(statuses),
             log=np.array([(e, k, r) for e, lg in enumerate(logs) for k, r in lg],
                          dtype=np.int64).reshape(-1, 3),
             state=state)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    # python tests/_dist_workers.py <worker> <rank> <world> <port> <out_dir> [arg]
    fn = globals()[sys.argv[1]]
    fn(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), *sys.argv[5:])
