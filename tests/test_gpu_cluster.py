"""The multi-GPU data path on the device (include/tbe_cluster.h): the routing partition,
pack and gather kernels and the key directory, each against its host mirror in
cluster.py (the code path the world-size-2 gloo tests drive), plus route_batch end to end
through RCCL at world size 1 with the HIP engine deciding."""
import os
import socket

import numpy as np
import pytest

from oracle import cref

pytestmark = pytest.mark.gpu


def _keys(n, seed, hot=0.0):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 1 << 40, n, dtype=np.uint64)
    if hot:
        pool = rng.integers(0, 1 << 40, 50, dtype=np.uint64)
        k = np.where(rng.random(n) < hot, pool[rng.integers(0, 50, n)], k)
    return k


@pytest.mark.parametrize("n_owners", [1, 2, 3, 8, 64, 256])
@pytest.mark.parametrize("n", [1, 4095, 4097, 300_000])
def test_route_plan_matches_host(engine_lib, gpu, n_owners, n):
    import torch
    from distributedratelimiting.redis_amd import _capi, cluster
    lib = _capi.load()
    k = _keys(n, n_owners * 7 + n, hot=0.3)
    dk = torch.from_numpy(k.view(np.int64)).to(gpu)
    pos = torch.empty(n, dtype=torch.int32, device=gpu)
    counts = torch.empty(n_owners, dtype=torch.int64, device=gpu)
    work = torch.empty(lib.tbe_route_workspace_bytes(n, n_owners), dtype=torch.uint8, device=gpu)
    assert lib.tbe_route_plan_device(dk.data_ptr(), n, n_owners, work.data_ptr(), pos.data_ptr(),
                                     counts.data_ptr(), None) == 0
    owner = cluster.key_owner(k, n_owners)
    assert all(lib.tbe_key_owner(int(x), n_owners) == o for x, o in zip(k[:200].tolist(), owner[:200].tolist()))
    order = np.argsort(owner, kind="stable")
    want = np.empty(n, dtype=np.int64)
    want[order] = np.arange(n)
    torch.cuda.synchronize()
    assert np.array_equal(pos.cpu().numpy().astype(np.int64), want)
    assert np.array_equal(counts.cpu().numpy(), np.bincount(owner, minlength=n_owners))
    # pack (send buffer) and gather (replies back to arrival order)
    p = torch.from_numpy(np.arange(n, dtype=np.int32) % 7).to(gpu)
    t = torch.from_numpy(np.arange(n, dtype=np.int64) * 3).to(gpu)
    send = torch.empty((n, 3), dtype=torch.int64, device=gpu)
    assert lib.tbe_route_pack_device(pos.data_ptr(), n, dk.data_ptr(), p.data_ptr(), t.data_ptr(),
                                     send.data_ptr(), None) == 0
    back = torch.empty_like(send)
    assert lib.tbe_route_gather_device(pos.data_ptr(), n, send.data_ptr(), 3, back.data_ptr(), None) == 0
    torch.cuda.synchronize()
    s = send.cpu().numpy()
    assert np.array_equal(s[:, 0].view(np.uint64), k[order]) and np.array_equal(s[:, 2], np.arange(n)[order] % 7)
    b = back.cpu().numpy()
    assert np.array_equal(b[:, 0].view(np.uint64), k) and np.array_equal(b[:, 1], np.arange(n) * 3)


@pytest.mark.parametrize("n_owners", [2, 8, 256])
@pytest.mark.parametrize("n", [4095, 300_000])
def test_route_plan_owner_map_matches_host(engine_lib, gpu, n_owners, n):
    """tbe_route_plan_map_device (owner = map[vnode(key)]) against the host mirror, for a
    balanced map of the batch's own loads and a random map; tbe_vnode_count_device against
    numpy's vnode histogram."""
    import torch
    from distributedratelimiting.redis_amd import _capi, cluster
    lib = _capi.load()
    k = _keys(n, n_owners * 11 + n, hot=0.3)
    dk = torch.from_numpy(k.view(np.int64)).to(gpu)
    loads = np.bincount(cluster.key_vnode(k), minlength=cluster.OWNER_MAP_SIZE)
    side = torch.cuda.Stream(gpu)
    with torch.cuda.stream(side):
        got_loads = cluster.vnode_loads(dk).cpu().numpy()
    assert np.array_equal(got_loads, loads)
    rng = np.random.default_rng(n)
    for omap in (cluster.balanced_owner_map(loads, n_owners),
                 rng.integers(0, n_owners, cluster.OWNER_MAP_SIZE).astype(np.uint8)):
        dmap = torch.from_numpy(omap).to(gpu)
        pos = torch.empty(n, dtype=torch.int32, device=gpu)
        counts = torch.empty(n_owners, dtype=torch.int64, device=gpu)
        work = torch.empty(lib.tbe_route_workspace_bytes(n, n_owners), dtype=torch.uint8, device=gpu)
        assert lib.tbe_route_plan_map_device(dk.data_ptr(), n, n_owners, dmap.data_ptr(), work.data_ptr(),
                                             pos.data_ptr(), counts.data_ptr(), None) == 0
        owner = cluster.key_owner(k, n_owners, omap)
        order = np.argsort(owner, kind="stable")
        want = np.empty(n, dtype=np.int64)
        want[order] = np.arange(n)
        torch.cuda.synchronize()
        assert np.array_equal(pos.cpu().numpy().astype(np.int64), want)
        assert np.array_equal(counts.cpu().numpy(), np.bincount(owner, minlength=n_owners))


def test_route_plan_bad_owner_map_is_bounds_safe(engine_lib, gpu):
    """a device owner map with entries >= n_owners is clamped to n_owners - 1 in
    the route kernels (include/tbe_cluster.h), so every position stays inside [0, n) and
    every count inside the n_owners array -- never an out-of-bounds write."""
    import torch
    from distributedratelimiting.redis_amd import _capi, cluster
    lib = _capi.load()
    n, n_owners = 100_000, 4
    k = _keys(n, 77, hot=0.1)
    dk = torch.from_numpy(k.view(np.int64)).to(gpu)
    bad = np.full(cluster.OWNER_MAP_SIZE, 200, dtype=np.uint8)
    bad[::3] = 1
    dmap = torch.from_numpy(bad).to(gpu)
    pos = torch.empty(n, dtype=torch.int32, device=gpu)
    counts = torch.zeros(n_owners + 8, dtype=torch.int64, device=gpu)   # guard words past n_owners
    work = torch.empty(lib.tbe_route_workspace_bytes(n, n_owners), dtype=torch.uint8, device=gpu)
    assert lib.tbe_route_plan_map_device(dk.data_ptr(), n, n_owners, dmap.data_ptr(), work.data_ptr(),
                                         pos.data_ptr(), counts.data_ptr(), None) == 0
    torch.cuda.synchronize()
    clamped = np.minimum(bad, n_owners - 1)
    owner = cluster.key_owner(k, n_owners, clamped)
    order = np.argsort(owner, kind="stable")
    want = np.empty(n, dtype=np.int64)
    want[order] = np.arange(n)
    assert np.array_equal(pos.cpu().numpy().astype(np.int64), want)
    c = counts.cpu().numpy()
    assert np.array_equal(c[:n_owners], np.bincount(owner, minlength=n_owners)) and not c[n_owners:].any()


def test_directory_matches_host(engine_lib, gpu):
    import torch
    with torch.cuda.stream(torch.cuda.Stream(gpu)):   # the device path needs a real stream
        _directory_matches_host(gpu)


def _directory_matches_host(gpu):
    import torch
    from distributedratelimiting.redis_amd import TbeError, cluster
    cap = 100_000                                                   # > the 90k key space: no overflow
    dd = cluster.DeviceDirectory(cap, device=0)
    hd = cluster.HostDirectory(cap)
    for b in range(5):
        k = _keys(40_000, 100 + b, hot=0.5) % np.uint64(90_000)       # repeats within and across batches
        got = dd.assign(torch.from_numpy(k.view(np.int64)).to(gpu)).cpu().numpy().view(np.uint64)
        assert np.array_equal(got, hd.assign(k)), b
    assert dd.size() == hd.size() == len(np.unique(np.concatenate(
        [_keys(40_000, 100 + b, hot=0.5) % np.uint64(90_000) for b in range(5)])))
    probe = np.array([1 << 50, 3, 1 << 51], np.uint64)
    lk = dd.lookup(torch.from_numpy(probe.view(np.int64)).to(gpu)).cpu().numpy().view(np.uint64)
    assert np.array_equal(lk, hd.lookup(probe))
    assert lk[0] == cluster.NO_ID and lk[2] == cluster.NO_ID
    # capacity: exact while the new keys of a batch fit; an over-capacity batch gives
    # unique ids in [0, capacity) to at most `capacity` keys and size() reports it
    small = cluster.DeviceDirectory(1000, device=0)
    hs = cluster.HostDirectory(1000)
    k = np.arange(900, dtype=np.uint64) * np.uint64(7919)
    first = small.assign(torch.from_numpy(k.view(np.int64)).to(gpu)).cpu().numpy().view(np.uint64)
    assert np.array_equal(first, hs.assign(k)) and small.size() == 900
    k = np.arange(3000, dtype=np.uint64) * np.uint64(7919) + np.uint64(5)
    got = small.assign(torch.from_numpy(k.view(np.int64)).to(gpu)).cpu().numpy().view(np.uint64)
    ok = got[got != cluster.NO_ID]
    assert ok.size <= 100 and np.unique(ok).size == ok.size and (ok < 1000).all()
    assert not set(ok.tolist()) & set(first.tolist())
    with pytest.raises(TbeError):
        small.size()


def cluster_error():
    from distributedratelimiting.redis_amd import TbeError
    return TbeError


def test_route_cancel_device_world1(engine_lib, gpu):
    """Queued waits routed through the device path and canceled through route_cancel with
    a DeviceDirectory (RCCL, world size 1) against the Python restatement."""
    import torch
    import torch.distributed as dist
    from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, cluster
    from oracle.semantics import QueueingTokenBucketTable, TokenBucketConfig
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    side = torch.cuda.Stream(gpu)
    try:
        torch.cuda.set_stream(side)
        n_keys, tl, ql = 64, 3, 5
        eng = QueueingTokenBucketEngine(n_keys, tl, 1, 10_000_000, ql, 0, device=0)
        dd = cluster.DeviceDirectory(n_keys, device=0)
        hd = cluster.HostDirectory(n_keys)
        ref = QueueingTokenBucketTable(TokenBucketConfig.from_options(tl, 1, 10_000_000), ql, 0)
        rng = np.random.default_rng(5)
        next_id = [0]

        def wait(lk, lp, lt):
            m = lk.numel()
            st = torch.empty(m, dtype=torch.uint8, device=gpu)
            rem = torch.empty(m, dtype=torch.int32, device=gpu)
            eng.wait_batch_device(lk, lp, lt, st, rem, next_id[0], stream=side.cuda_stream)
            ids = next_id[0] + torch.arange(m, dtype=torch.int64, device=gpu)
            next_id[0] += m
            return st, rem, ids

        def cancel(lk, ids):
            assert lk.is_cuda and ids.is_cuda
            eng.synchronize()
            return eng.cancel(lk.cpu().numpy().view(np.uint64), ids.cpu().numpy())

        hits = 0
        for b in range(3):
            n = 400
            k = (rng.integers(0, 40, n) * 7919 + 11).astype(np.uint64)
            p = rng.choice([1, 1, 2, 3], n).astype(np.int32)
            t = (1_760_000_000_000_000 + b * 600_000 + np.sort(rng.integers(0, 1000, n))).astype(np.int64)
            st, rem, ids = cluster.route_batch(wait, torch.from_numpy(k.view(np.int64)).to(gpu),
                                               torch.from_numpy(p).to(gpu), torch.from_numpy(t).to(gpu), dd)
            hk = hd.assign(k)
            base = b * n
            exp = [ref.acquire(int(hk[i]), int(p[i]), int(t[i]), base + i) for i in range(n)]
            assert st.cpu().numpy().tolist() == [e[0] for e in exp], b
            assert rem.cpu().numpy().tolist() == [e[1] for e in exp], b
            assert ids.cpu().numpy().tolist() == list(range(base, base + n))
            pick = np.array([i for i in range(n) if i % 3 == 0 or i % 41 == 7])
            hit = cluster.route_cancel(cancel, torch.from_numpy(k[pick].view(np.int64)).to(gpu),
                                       ids[torch.from_numpy(pick).to(gpu)], dd)
            want = [int(ref.cancel(int(hk[i]), base + int(i))) for i in pick]
            assert hit.cpu().numpy().tolist() == want, b
            hits += sum(want)
            lk, li, lr = eng.refresh(1_760_000_000_000_000 + b * 600_000 + 500_000)
            exp_log = ref.refresh(1_760_000_000_000_000 + b * 600_000 + 500_000)
            assert list(zip(lk.tolist(), li.tolist(), lr.tolist())) == [tuple(e) for e in exp_log], b
        assert hits > 0
        with pytest.raises(TypeError):    # a DeviceDirectory takes device tensors only
            cluster.route_cancel(cancel, np.zeros(2, np.uint64), np.zeros(2, np.int64), dd)
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(gpu))
        dist.destroy_process_group()


def test_route_batch_device_world1(engine_lib, gpu):
    """route_batch's device path (route kernels + RCCL all-to-all + directory + the HIP
    engine) at world size 1, against the C restatement on the directory's dense ids."""
    import torch
    import torch.distributed as dist
    from distributedratelimiting.redis_amd import TokenBucketEngine, cluster, fill_rate
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    side = torch.cuda.Stream(gpu)   # the device path orders its kernels on a real (non-NULL) stream
    try:
        torch.cuda.set_stream(side)
        cap = 400_000  # > distinct keys over the 3 batches (~330k)
        eng = TokenBucketEngine(cap, 5, 2, 10_000_000, device=0)
        dd = cluster.DeviceDirectory(cap, device=0)
        hd = cluster.HostDirectory(cap)
        ref = cref.CTokenBucket(cap, 5, fill_rate(2, 10_000_000))
        rng = np.random.default_rng(2)

        def decide(lk, lp, lt):
            g = torch.empty(lk.numel(), dtype=torch.uint8, device=gpu)
            r = torch.empty(lk.numel(), dtype=torch.int32, device=gpu)
            eng.acquire_batch_device(lk, lp, lt, g, r, stream=torch.cuda.current_stream(gpu).cuda_stream)
            return g, r

        for b in range(3):
            n = 150_000
            k = (_keys(n, 9 + b, hot=0.2) % np.uint64(1 << 20)).astype(np.uint64)
            p = rng.integers(0, 4, n).astype(np.int32)
            t = (1_760_000_000_000_000 + b * 900_000 + np.sort(rng.integers(0, 900_000, n))).astype(np.int64)
            g, r = cluster.route_batch(decide, torch.from_numpy(k.view(np.int64)).to(gpu), torch.from_numpy(p).to(gpu),
                                       torch.from_numpy(t).to(gpu), dd)
            ids = hd.assign(k)
            assert not hd.overflow
            g_ref, r_ref = ref.acquire_batch(ids, p, t)
            assert np.array_equal(g.cpu().numpy(), g_ref) and np.array_equal(r.cpu().numpy(), r_ref), b
        # int64 permits (the host API's natural type) are converted, not misread
        k = (_keys(5000, 77, hot=0.2) % np.uint64(1 << 20)).astype(np.uint64)
        p = rng.integers(0, 4, 5000)
        t = (1_760_000_000_000_000 + 3 * 900_000 + np.sort(rng.integers(0, 900_000, 5000))).astype(np.int64)
        g, r = cluster.route_batch(decide, torch.from_numpy(k.view(np.int64)).to(gpu), torch.from_numpy(p).to(gpu),
                                   torch.from_numpy(t).to(gpu), dd)
        g_ref, r_ref = ref.acquire_batch(hd.assign(k), p.astype(np.int32), t)
        assert np.array_equal(g.cpu().numpy(), g_ref) and np.array_equal(r.cpu().numpy(), r_ref)
        # a batch bringing more new keys than ids remain raises before any decision
        small = cluster.DeviceDirectory(1000, device=0)
        calls = []
        with pytest.raises(cluster_error()):
            cluster.route_batch(lambda *a: calls.append(1) or decide(*a),
                                torch.arange(1500, dtype=torch.int64, device=gpu),
                                torch.ones(1500, dtype=torch.int32, device=gpu),
                                torch.full((1500,), 1_760_000_000_000_000, dtype=torch.int64, device=gpu), small)
        assert not calls
        # strict=False (bench.py --route timed): no synchronisation per batch; the engine
        # refuses the overflowing batch itself (keys beyond capacity get no id) and the next
        # check raises TBE_ERANGE
        lax = cluster.DeviceDirectory(1000, device=0, strict=False)
        eng2 = TokenBucketEngine(1000, 5, 2, 10_000_000, device=0)

        def decide2(lk, lp, lt):
            g = torch.empty(lk.numel(), dtype=torch.uint8, device=gpu)
            r = torch.empty(lk.numel(), dtype=torch.int32, device=gpu)
            eng2.acquire_batch_device(lk, lp, lt, g, r, stream=torch.cuda.current_stream(gpu).cuda_stream)
            return g, r
        cols = (torch.ones(1500, dtype=torch.int32, device=gpu),
                torch.full((1500,), 1_760_000_000_000_000, dtype=torch.int64, device=gpu))
        cluster.route_batch(decide2, torch.arange(1500, dtype=torch.int64, device=gpu), *cols, lax)
        with pytest.raises(cluster_error()):
            eng2.synchronize()                                # the batch with id-less keys was refused
        torch.cuda.synchronize()
        with pytest.raises(cluster_error()):
            cluster.route_batch(decide2, torch.arange(1500, 3000, dtype=torch.int64, device=gpu), *cols, lax)
        eng2.close()
        lax.close()
        with pytest.raises(ValueError):                       # the NULL default stream is refused
            torch.cuda.set_stream(torch.cuda.default_stream(gpu))
            cluster.route_batch(decide, torch.zeros(4, dtype=torch.int64, device=gpu),
                                torch.ones(4, dtype=torch.int32, device=gpu),
                                torch.zeros(4, dtype=torch.int64, device=gpu), dd)
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream(gpu))
        dist.destroy_process_group()
