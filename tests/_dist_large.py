"""Rank bodies of tests/test_gpu_dist_large.py: the sharded path at sizes that exercise it
(VERDICT r03 item 1).  TEST INFRASTRUCTURE: the references are the C restatement
(oracle/tb_ref.c through oracle/cref.py).

Two rank processes share the test box's GPU over gloo (RCCL refuses two ranks on one
device; cluster.py stages the device path's collectives through host memory), each with
its own HIP engine and device key directory.  Every rank generates every rank's share of
the global request stream (the device generators are deterministic), so it can run the
serial reference of the WHOLE stream itself -- per step, rank 0's batch, then rank 1's
(PTB:42: one key space; the per-key order route_batch promises) -- and compare its own
replies, drain logs and the rows of the keys it owns.  Results go to a small npz of
mismatch counts and statistics that the test asserts on.

* tb_large_worker: config C's form -- one global Zipf(1.1) stream over 2^24 keys, 2^22
  requests per rank per step, 4 steps (hot-key runs active on the owners from the third
  batch) -- or config B's uniform stream of the same size; routed before the steps
  (bench.py --route pre: route_requests, decide, route_replies afterwards) or inside
  every step (cluster.route_batch).
* q_large_worker: queued waits over 2^17 keys (QueueLimit 16, TokenLimit 4), 2^18
  requests per rank per step, routed, a share of them canceled through route_cancel,
  then a replenish tick on every owner (Q:67-134, Q:480-506, Q:237-271).
* ap_large_worker: two approximate clients over 2^17 shared keys with queued waits and
  local cancels, refresh epochs in both exchange modes (A:116-214, A:412-508, A:241-270).
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tests._dist_workers import _hip_setup, _init  # noqa: E402

T0_US = 1_760_000_000_000_000
REF_THREADS = 8


def _save(out_dir, name, **kw):
    np.savez(os.path.join(out_dir, name), **{k: np.asarray(v) for k, v in kw.items()})


# ------------------------------------------------------------------ token bucket, 2^24 keys
TBL = dict(n_keys=1 << 24, n=1 << 22, steps=4, token_limit=10, tokens_per_period=1,
           period_ticks=10_000_000, interval_us=10_000, seed_zipf=0x5EED000C, seed_uniform=0x5EED000B)


def tb_large_worker(rank: int, world: int, port: int, out_dir: str, keyspace: str, route_mode: str,
                    map_kind: str = "hash"):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import TokenBucketEngine, _capi, cluster, fill_rate
    from oracle import cref

    C = TBL
    K, N, S = C["n_keys"], C["n"], C["steps"]
    lib = _capi.load()
    seed = C["seed_zipf"] if keyspace == "zipf" else C["seed_uniform"]
    sh = stream.cuda_stream

    def gen(step, src):   # rank src's share of the global stream at `step` (bench.py's draw order)
        g0 = (step * world + src) * N
        k = torch.empty(N, dtype=torch.int64, device=dev)
        p = torch.empty(N, dtype=torch.int32, device=dev)
        t = torch.empty(N, dtype=torch.int64, device=dev)
        assert lib.tbe_gen_batch_device(seed, K, g0, N, 1, 2, T0_US + step * C["interval_us"], C["interval_us"],
                                        k.data_ptr(), p.data_ptr(), t.data_ptr(), sh) == 0
        if keyspace == "zipf":
            assert lib.tbe_gen_zipf_keys_device(seed, K, 1.1, g0, N, k.data_ptr(), sh) == 0
        return k, p, t

    omap = None
    if map_kind == "balanced":
        # the owner map every rank builds from the all-reduced virtual-node loads of step 0
        loads = cluster.vnode_loads(gen(0, rank)[0])
        cluster._all_reduce_sum(loads)
        omap = cluster.balanced_owner_map(loads.cpu().numpy(), world, n_keys=K)
    cap = cluster.keys_per_rank(K, world, owner_map=omap)
    eng = TokenBucketEngine(cap, C["token_limit"], C["tokens_per_period"], C["period_ticks"], device=0,
                            stage_timing=True, max_batch=2 * N)
    directory = cluster.DeviceDirectory(cap, device=0)

    def decide(lk, lp, lt):
        g = torch.empty(lk.numel(), dtype=torch.uint8, device=dev)
        r = torch.empty(lk.numel(), dtype=torch.int32, device=dev)
        eng.acquire_batch_device(lk, lp, lt, g, r, stream=sh)
        return g, r

    own = [gen(s, rank) for s in range(S)]
    replies = []
    if route_mode == "pre":
        # bench.py --route pre: every step's requests reach their owners before any is
        # decided (ingest partitioned); the replies travel back afterwards, for the check
        routed = [cluster.route_requests(*own[s], directory, owner_map=omap) for s in range(S)]
        cols = [decide(*routed[s][0]) for s in range(S)]
        for s in range(S):
            out = cluster.route_replies(routed[s][1], cols[s])
            replies.append((out[0].to(torch.uint8).cpu().numpy(), out[1].to(torch.int32).cpu().numpy()))
        recv = [int(routed[s][0][0].numel()) for s in range(S)]
    else:
        recv = []
        for s in range(S):
            g, r = cluster.route_batch(decide, *own[s], directory, owner_map=omap)
            replies.append((g.cpu().numpy(), r.cpu().numpy()))
    eng.synchronize()
    stages = eng.stage_times()
    layout = eng.layout()
    del own

    # the serial reference of the whole stream, step by step
    ref = cref.CTokenBucket(K, C["token_limit"], fill_rate(C["tokens_per_period"], C["period_ticks"]))
    mism_g, mism_r, load, max_mult, owned = [], [], [], [], []
    for s in range(S):
        bs = [tuple(x.cpu().numpy() for x in gen(s, src)) for src in range(world)]
        k = np.concatenate([b[0] for b in bs]).view(np.uint64)
        p = np.concatenate([b[1] for b in bs])
        t = np.concatenate([b[2] for b in bs])
        g_ref, r_ref = ref.acquire_batch(k, p, t, threads=REF_THREADS)
        mine = slice(rank * N, (rank + 1) * N)
        mism_g.append(int((replies[s][0] != g_ref[mine]).sum()))
        mism_r.append(int((replies[s][1] != r_ref[mine]).sum()))
        mk = k[cluster.key_owner(k, world, omap) == rank]
        _, cnt = np.unique(mk, return_counts=True)
        load.append(int(mk.size))
        max_mult.append(int(cnt.max()) if cnt.size else 0)
        owned.append(np.unique(mk))
        if route_mode != "pre":
            recv.append(int(mk.size))
    owned = np.unique(np.concatenate(owned))
    ids = directory.lookup(torch.from_numpy(owned.view(np.int64)).to(dev)).cpu().numpy()
    v, tt = eng.export_state()
    v_ref, t_ref = ref.export_state()
    tab_t = int((tt[ids] != t_ref[owned]).sum())
    tab_v = int((v[ids].view(np.uint64) != v_ref[owned].view(np.uint64)).sum())
    rest = np.ones(cap, dtype=bool)
    rest[ids] = False
    stray = int((tt[rest] != np.iinfo(np.int64).min).sum())    # rows no owned key maps to stay absent
    g_last = replies[-1][0]
    _save(out_dir, f"tbl_{keyspace}_{route_mode}_{map_kind}_{rank}.npz", mism_g=mism_g, mism_r=mism_r, tab_t=tab_t,
          tab_v=tab_v, stray=stray, n_owned=owned.size, ids_unique=np.unique(ids).size,
          ids_in_range=int((ids < cap).all()), load=load, recv=recv, max_mult=max_mult,
          hot_ms=stages.get("hot", 0.0), passes=layout["passes"], grant_last=float(g_last.mean()),
          n=N, steps=S)
    eng.close()
    directory.close()
    ref.close()
    dist.barrier()
    dist.destroy_process_group()


# ------------------------------------------------------------------ queued waits, 2^17 keys
QL = dict(n_keys=1 << 17, n=1 << 18, steps=3, token_limit=4, tokens_per_period=1, period_ticks=10_000_000,
          queue_limit=16)


def q_large_batch(src: int, step: int):
    rng = np.random.default_rng(9000 + 100 * src + step)
    n = QL["n"]
    keys = rng.integers(0, QL["n_keys"], n, dtype=np.uint64)
    permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
    ts = T0_US + step * 700_000 + np.sort(rng.integers(0, 1_000, n))
    return keys, permits, ts.astype(np.int64)


def q_large_pick(st_ref: np.ndarray) -> np.ndarray:
    """A third of the queued requests, plus some that are not queued."""
    i = np.arange(st_ref.size)
    return np.flatnonzero(((i % 3 == 0) & (st_ref == 2)) | (i % 97 == 5))


def q_tick_ts(step: int) -> int:
    return T0_US + step * 700_000 + 500_000


def q_large_worker(rank: int, world: int, port: int, out_dir: str, order: str):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, cluster, fill_rate
    from oracle import cref

    order = int(order)
    C = QL
    K, N, S = C["n_keys"], C["n"], C["steps"]
    sh = stream.cuda_stream
    cap = cluster.keys_per_rank(K, world)
    eng = QueueingTokenBucketEngine(cap, C["token_limit"], C["tokens_per_period"], C["period_ticks"],
                                    C["queue_limit"], order, device=0, max_batch=2 * N)
    directory = cluster.DeviceDirectory(cap, device=0)
    ref = cref.CQueueingTokenBucket(K, C["token_limit"], fill_rate(C["tokens_per_period"], C["period_ticks"]),
                                    C["queue_limit"], order)
    next_id = [0]
    owner_evicted = []

    def wait(lk, lp, lt):   # the owner's engine: WaitAsync, ids assigned in arrival order
        m = lk.shape[0]
        base = next_id[0]
        next_id[0] += m
        st = torch.empty(m, dtype=torch.uint8, device=dev)
        rem = torch.empty(m, dtype=torch.int32, device=dev)
        if m:
            eng.wait_batch_device(lk, lp, lt, st, rem, base, wait=True, stream=sh)
            if order == 1:
                owner_evicted.append(eng.evicted()[1].copy())
        return st, rem, base + torch.arange(m, dtype=torch.int64, device=dev)

    def cancel(lk, ids):
        eng.synchronize()
        return eng.cancel(lk.cpu().numpy().view(np.uint64), ids.cpu().numpy())

    ref_id = lambda s, src, i: (s * world + src) * N + i   # noqa: E731
    key_of_ref = {}
    res = dict(mism_st=[], mism_rem=[], mism_hit=[], mism_log=[], mism_ev=[], hits=[], log_len=[], queued=[])
    to_ref = {}    # this owner's request id -> reference id
    gkey_of_local = {}
    for s in range(S):
        bs = [q_large_batch(src, s) for src in range(world)]
        for src, (k, _, _) in enumerate(bs):
            key_of_ref[(s, src)] = k
        # the owner's received order: per source rank, its requests for this owner in arrival order
        base = next_id[0]
        got = [np.flatnonzero(cluster.key_owner(k, world) == rank) for (k, _, _) in bs]
        j = 0
        for src, idx in enumerate(got):
            for i in idx.tolist():
                to_ref[base + j] = ref_id(s, src, i)
                j += 1
        k, p, t = bs[rank]
        kd, pd, tdv = (torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev) for x in (k, p, t))
        owner_evicted.clear()
        st, rem, ids = (x.cpu().numpy() for x in cluster.route_batch(wait, kd, pd, tdv, directory))
        # reference: rank 0's batch, then rank 1's
        ev_ref = []
        st_refs = []
        for src, (kk, pp, tt) in enumerate(bs):
            st_r, rem_r, _, evid = ref.acquire_batch(kk, pp, tt, ref_id(s, src, 0))
            st_refs.append(st_r)
            ev_ref.append(evid)
            if src == rank:
                res["mism_st"].append(int((st != st_r).sum()))
                res["mism_rem"].append(int((rem != rem_r).sum()))
                res["queued"].append(int((st_r == 2).sum()))
        # evictions (NewestFirst): the owner's evicted ids = the reference's evicted ids of
        # the keys it owns
        if order == 1:
            evr = np.concatenate(ev_ref)
            ev_keys = np.array([key_of_ref[(int(x) // N // world, int(x) // N % world)][int(x) % N] for x in evr.tolist()],
                               dtype=np.uint64)
            want = np.sort(evr[cluster.key_owner(ev_keys, world) == rank]) if evr.size else evr
            mine_ev = np.sort(np.array([to_ref[int(x)] for x in np.concatenate(owner_evicted).tolist()], np.int64)) \
                if owner_evicted else np.zeros(0, np.int64)
            res["mism_ev"].append(int(want.size != mine_ev.size or not np.array_equal(want, mine_ev)))
        # cancels: every source cancels the picks of its batch (chosen from the reference's
        # statuses, so every rank knows every source's picks), routed to the owners
        picks = [q_large_pick(st_refs[src]) for src in range(world)]
        my = picks[rank]
        hit = cluster.route_cancel(cancel, torch.from_numpy(k[my].view(np.int64)).to(dev),
                                   torch.from_numpy(ids[my].astype(np.int64)).to(dev), directory).cpu().numpy()
        for src in range(world):
            kk = bs[src][0]
            want = ref.cancel(kk[picks[src]], ref_id(s, src, 0) + picks[src].astype(np.int64))
            if src == rank:
                res["mism_hit"].append(int((hit != want).sum()))
                res["hits"].append(int(want.sum()))
        # the replenish tick on every owner vs the reference tick, restricted to owned keys
        lk, li, lr = eng.refresh(q_tick_ts(s))
        rk, ri, rr = ref.refresh(q_tick_ts(s))
        sel = cluster.key_owner(rk, world) == rank
        rk, ri, rr = rk[sel], ri[sel], rr[sel]
        need = np.setdiff1d(np.unique(lk), np.array(list(gkey_of_local.keys()), dtype=np.uint64))
        if need.size:
            # local id -> global key: the owned keys seen so far, looked up in the directory
            seen = np.unique(np.concatenate([key_of_ref[(s2, src)] for s2 in range(s + 1) for src in range(world)]))
            seen = seen[cluster.key_owner(seen, world) == rank]
            lid = directory.lookup(torch.from_numpy(seen.view(np.int64)).to(dev)).cpu().numpy()
            gkey_of_local.update(zip(lid.tolist(), seen.tolist()))
        gk = np.array([gkey_of_local[int(x)] for x in lk.tolist()], dtype=np.uint64)
        gi = np.array([to_ref[int(x)] for x in li.tolist()], dtype=np.int64)
        o = np.argsort(gk, kind="stable")
        same = (gk.size == rk.size and np.array_equal(gk[o], rk) and np.array_equal(gi[o], ri)
                and np.array_equal(lr[o], rr))
        res["mism_log"].append(0 if same else 1)
        res["log_len"].append(int(rk.size))
    # final rows and queues of the owned keys
    seen = np.unique(np.concatenate(list(key_of_ref.values())))
    seen = seen[cluster.key_owner(seen, world) == rank]
    lid = directory.lookup(torch.from_numpy(seen.view(np.int64)).to(dev)).cpu().numpy()
    v, tt = eng.export_state()
    v_ref, t_ref = ref.bucket_state()
    tab = int((tt[lid] != t_ref[seen]).sum() + (v[lid].view(np.uint64) != v_ref[seen].view(np.uint64)).sum())
    qm = 0
    for j in range(0, seen.size, max(1, seen.size // 3000)):
        mine = [(to_ref[i], p) for i, p in eng.queue_of(int(lid[j]))]
        qm += int(mine != ref.queue_of(int(seen[j])))
    _save(out_dir, f"ql_{order}_{rank}.npz", tab=tab, queues=qm, n_owned=seen.size, **res)
    eng.close()
    directory.close()
    ref.close()
    dist.barrier()
    dist.destroy_process_group()


# ------------------------------------------------------------------ approximate, 2^17 keys
APL = dict(n_keys=1 << 17, n=1 << 18, epochs=4, token_limit=20, tokens_per_period=10, period_ticks=10_000_000,
           queue_limit=8)


def ap_large_batch(client: int, epoch: int):
    rng = np.random.default_rng(31000 + 101 * client + epoch)
    n = APL["n"]
    return (rng.integers(0, APL["n_keys"], n, dtype=np.uint64),
            rng.choice([0, 1, 1, 2, 3, 5], n).astype(np.int32))


def ap_epoch_ts(epoch: int) -> int:
    return T0_US + (epoch + 1) * 1_000_000 + epoch * 37_000


def ap_large_worker(rank: int, world: int, port: int, out_dir: str, mode: str, order: str = "0"):
    dist = _init(rank, world, port)
    torch, dev, stream = _hip_setup()
    from distributedratelimiting.redis_amd import ApproximateEngine, cluster
    from oracle import cref

    order = int(order)
    C = APL
    K, N, E = C["n_keys"], C["n"], C["epochs"]
    eng = ApproximateEngine(K, C["token_limit"], C["tokens_per_period"], C["period_ticks"], C["queue_limit"], order,
                            device=0, max_batch=N)
    # every client's reference (each rank can generate every client's batches): the clients'
    # local tiers and their replicas of the global tier
    refs = [cref.CApprox(K, C["token_limit"], C["tokens_per_period"], C["period_ticks"], C["queue_limit"], order)
            for _ in range(world)]
    stagger = 1_000_000 // world
    res = dict(mism_st=[], mism_av=[], mism_ev=[], mism_hit=[], mism_log=[], queued=[], hits=[], log_len=[])
    for e in range(E):
        rid = e * N
        for c in range(world):
            keys, permits = ap_large_batch(c, e)
            st_r, av_r, ca_r, ev_r = refs[c].acquire_batch(keys, permits, wait=True, id_base=rid, threads=REF_THREADS)
            if c == rank:
                st, av, (ca, ev) = eng.acquire_batch(keys, permits, wait=True, id_base=rid)
                res["mism_st"].append(int((st != st_r).sum()))
                res["mism_av"].append(int((av != av_r).sum()))
                res["mism_ev"].append(int(not (np.array_equal(ca, ca_r) and np.array_equal(ev, ev_r))))
                res["queued"].append(int((st_r == 2).sum()))
            # local cancels (CancelQueueState, A:531-557): a fifth of the queued requests
            pick = np.flatnonzero((st_r == 2) & (np.arange(N) % 5 == 0))
            want = refs[c].cancel(keys[pick], rid + pick.astype(np.int64))
            if c == rank:
                hit = eng.cancel(keys[pick], rid + pick.astype(np.int64))
                res["mism_hit"].append(int((hit != want).sum()))
                res["hits"].append(int(want.sum()))
        counts = torch.zeros(K, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        lk, li, lr = cluster.approx_epoch(eng, counts, ap_epoch_ts(e), stagger, mode=mode)
        cr = [refs[c].collect() for c in range(world)]
        if mode == "clients":        # every rank a client: client c's sync sees clients < c (§8e option 2)
            allc = np.concatenate(cr)
            logs = [refs[c].sync(allc, world, c, ap_epoch_ts(e), stagger, threads=REF_THREADS) for c in range(world)]
        else:                        # the node is one client: the summed counts, one sync call per key
            tot = np.sum(np.stack(cr), axis=0).astype(np.int32)
            logs = [refs[c].sync(tot, 1, 0, ap_epoch_ts(e), 0, threads=REF_THREADS) for c in range(world)]
        rk, ri, rr = logs[rank]
        same = (np.array_equal(lk, rk) and np.array_equal(li, ri) and np.array_equal(lr, rr))
        res["mism_log"].append(0 if same else 1)
        res["log_len"].append(int(rk.size))
    x = refs[rank].export()
    v, p, t = eng.export_global()
    glob = int((v.view(np.uint64) != x["v"].view(np.uint64)).sum() + (p.view(np.uint64) != x["p"].view(np.uint64)).sum()
               + (t != x["t_us"]).sum())
    loc = 0
    for k in range(0, K, 61):
        lo, gl, est, av, q = eng.local_state(k)
        loc += int((lo, gl, est, av, q) != (int(x["local"][k]), int(x["global"][k]), float(x["est"][k]),
                                             int(x["available"][k]), int(x["queued"][k])))
        if k % 610 == 0:
            loc += int(eng.queue_of(k) != refs[rank].queue_of(k))
    _save(out_dir, f"apl_{mode}_{order}_{rank}.npz", glob=glob, loc=loc, **res)
    eng.close()
    for r in refs:
        r.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    # python tests/_dist_large.py <worker> <rank> <world> <port> <out_dir> [args...]
    fn = globals()[sys.argv[1]]
    fn(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), *sys.argv[5:])
