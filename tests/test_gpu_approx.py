"""GPU parity of the ApproximateTokenBucket path: N client engines on one GPU (counts
exchanged by concatenating their device buffers -- the all-gather RCCL performs across
GPUs) against N oracle clients sharing one oracle global tier (oracle/semantics.py
ApproxClient + ApproxGlobalTable, whose sync script is pinned by the Lua-replay golden
vectors)."""
import numpy as np
import pytest

from oracle.semantics import (NEWEST_FIRST, OLDEST_FIRST, ApproxClient, ApproxGlobalTable,
                              approx_refresh_all)

pytestmark = pytest.mark.gpu

S_US = 1_760_572_800 * 1_000_000


@pytest.mark.parametrize("n_clients,order,qlimit,wait,pack,limit", [
    (1, OLDEST_FIRST, 8, True, True, 20), (3, NEWEST_FIRST, 4, True, True, 20),
    (8, OLDEST_FIRST, 16, True, True, 20), (2, OLDEST_FIRST, 0, False, True, 20),
    # the SoA partition records (TBE_FLAG_NO_PACK; the default when key + permit code
    # leave less than 32 bits for the arrival index)
    (3, NEWEST_FIRST, 4, True, False, 20), (2, OLDEST_FIRST, 0, False, False, 20),
    # the reply widths' boundary: TokenLimit 16382 is the largest whose
    # AvailableTokens fit the two-byte replies (14 bits, 16383 = "no script call"); 16383
    # and above take four-byte replies
    (2, OLDEST_FIRST, 8, True, True, 16382), (2, NEWEST_FIRST, 8, True, True, 16383),
    (2, OLDEST_FIRST, 0, False, True, 16382),
    # 50k keys: two partition passes, so fold records (marked by a negative limit)
    (2, NEWEST_FIRST, 4, True, True, -20), (2, OLDEST_FIRST, 0, False, True, -20)])
def test_clients_epochs(engine_lib, gpu, n_clients, order, qlimit, wait, pack, limit):
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n, tokens, ticks = (300 if limit > 0 else 50_000), 4000, 10, 10_000_000
    limit = abs(limit)
    rng = np.random.default_rng(n_clients * 100 + order * 10 + qlimit + limit)
    engines = [ApproximateEngine(n_keys, limit, tokens, ticks, qlimit, order, device=0, pack=pack)
               for _ in range(n_clients)]
    assert engines[0].layout()["packed"] == pack
    assert engines[0].layout()["medium"] == (limit <= 16382)
    assert engines[0].layout()["passes"] == (1 if n_keys == 300 else 2)
    assert engines[0].layout()["fold_records"] == (pack and n_keys != 300)
    choices = [0, 1, 1, 2, 3, 25] + ([limit // 3, limit // 2, limit, limit + 1] if limit > 100 else [])
    clients = [ApproxClient(limit, tokens, ticks, qlimit, order) for _ in range(n_clients)]
    table = ApproxGlobalTable(clients[0].decay_rate)
    counts = [torch.zeros(n_keys, dtype=torch.int32, device=gpu) for _ in range(n_clients)]
    torch.cuda.synchronize()   # the engine's NULL-stream calls take inputs complete at the call
    rid = 0
    for epoch in range(6):
        for r in range(n_clients):
            keys = rng.integers(0, n_keys, n).astype(np.uint64)
            permits = rng.choice(choices, n).astype(np.int32)
            st, av, (cause, ids) = engines[r].acquire_batch(keys, permits, wait=wait, id_base=rid)
            exp = []
            for i, (k, p) in enumerate(zip(keys.tolist(), permits.tolist())):
                c = clients[r]
                if wait:
                    status, ev = c.wait(k, p, rid + i)
                else:
                    status, ev = c.acquire(k, p), []
                a = -1 if status == 3 else c.available(c.st(k))
                exp.append((status, a, ev))
            assert st.tolist() == [x[0] for x in exp]
            assert av.tolist() == [x[1] for x in exp]
            exp_ev = [(i, x) for i, e in enumerate(exp) for x in e[2]]
            assert list(zip(cause.tolist(), ids.tolist())) == exp_ev
            rid += n
        ts = S_US + epoch * 1_000_000 + int(rng.integers(0, 300_000))
        stagger = 1_000_000 // n_clients
        for r in range(n_clients):
            engines[r].collect(counts[r])
        allc = torch.cat(counts)
        torch.cuda.synchronize()   # the engines' sync replay reads allc on their own streams
        logs = [engines[r].sync(allc, n_clients, r, ts, stagger) for r in range(n_clients)]
        exp_logs = approx_refresh_all(clients, table, ts, stagger, range(n_keys))
        for r in range(n_clients):
            k, i, _ = logs[r]
            assert list(zip(k.tolist(), i.tolist())) == exp_logs[r]
        for r in range(n_clients):
            for key in range(0, n_keys, 7 if n_keys == 300 else 613):
                lo, gl, est, av, q = engines[r].local_state(key)
                s = clients[r].st(key)
                assert (lo, gl, est, av, q) == (s.local, s.global_, s.est, clients[r].available(s), len(s.queue))


def test_sync_stream_orders_after_producer(engine_lib, gpu):
    """tbe_approx_sync_stream orders the replay after the stream that
    produces the exchanged counts.  Here the counts are concatenated by torch.cat on a side
    stream behind a long spin, with no host synchronisation before the call; the replay
    must equal that of twin engines whose counts were complete at the call (A:439)."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n, clients = 200_000, 1 << 20, 3
    rng = np.random.default_rng(11)
    twins = [[ApproximateEngine(n_keys, 20, 10, 10_000_000, 4, 0, device=0) for _ in range(clients)]
             for _ in range(2)]
    counts = [[torch.zeros(n_keys, dtype=torch.int32, device=gpu) for _ in range(clients)] for _ in range(2)]
    side = torch.cuda.Stream(gpu)
    for epoch in range(3):
        batches = [rng.integers(0, n_keys, n).astype(np.uint64) for _ in range(clients)]
        for engs in twins:
            for r in range(clients):
                engs[r].acquire_batch(batches[r], np.ones(n, np.int32), wait=True, id_base=epoch * n)
        ts = S_US + epoch * 1_000_000
        for engs, cs in zip(twins, counts):
            for r in range(clients):
                engs[r].collect(cs[r])
        torch.cuda.synchronize()
        ref_all = torch.cat(counts[1])
        torch.cuda.synchronize()
        want = [twins[1][r].sync(ref_all, clients, r, ts, 1000) for r in range(clients)]
        with torch.cuda.stream(side):
            torch.cuda._sleep(200_000_000)              # the producer is still busy at the call
            allc = torch.cat(counts[0])
        got = [twins[0][r].sync(allc, clients, r, ts, 1000, stream=side.cuda_stream) for r in range(clients)]
        for g, w in zip(got, want):
            for a, b in zip(g, w):
                assert np.array_equal(a, b)
        for key in range(0, n_keys, 997):
            for r in range(clients):
                assert twins[0][r].local_state(key) == twins[1][r].local_state(key)
        side.synchronize()
    a, b = twins[0][0].export_global(), twins[1][0].export_global()
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64))


GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)),
                                    "golden")


@pytest.mark.parametrize("name", ["approx_one_client", "approx_eight_clients", "approx_slow_decay"])
def test_golden_sync_trace_on_gpu(engine_lib, gpu, name):
    """The reference's sync script replayed by Lua (tests/golden/make_golden.py): each
    recorded ScriptEvaluateAsync(_syncScript, {BucketId, LocalCount}) call (A:439) runs as
    one tbe_approx_sync on the device; _globalThrottleScore (A:441) and the estimate built
    from the "%.14g" period string (A:442-443) must match after every call, and the
    replica's final {v, p, t} must equal the script's hash (A:265)."""
    import os
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    from oracle.semantics import instance_count_estimate, new_t_of
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        g = {k: z[k] for k in z.files}
    ticks = int(g["period_ticks"])
    eng = ApproximateEngine(1, 1000, int(g["tokens_per_period"]), ticks, 0, 0, device=0)
    from distributedratelimiting.redis_amd import fill_rate
    assert fill_rate(int(g["tokens_per_period"]), ticks) == float(g["decay_rate"])
    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
    for i in range(len(g["counts"])):
        cnt.fill_(int(g["counts"][i]))
        torch.cuda.synchronize()
        eng.sync(cnt, 1, 0, int(g["ts_us"][i]), 0)
        _, gl, est, _, _ = eng.local_state(0)
        assert gl == int(g["global_score"][i]), i
        want = instance_count_estimate(ticks / 1e7, float(g["period"][i]))
        assert est == want or (est != est and want != want), (i, est, want)
    v, p, t = eng.export_global()
    assert (v[0], p[0], new_t_of(int(t[0]))) == (g["final_v"], g["final_p"], g["final_t"])


def test_numfmt_round_trip_on_device(engine_lib, gpu):
    """round_trip_14g as compiled for gfx950 (tbe_numfmt_device) == Python float("%.14g" % x)
    on the inputs of tests/test_numfmt.py (the CPU test compiles the same header with g++)."""
    import importlib.util
    import os
    import torch
    from distributedratelimiting.redis_amd import _capi
    spec = importlib.util.spec_from_file_location("_numfmt_cases", os.path.join(os.path.dirname(__file__),
                                                                                "test_numfmt.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    xs = np.array(mod.values() + [0.0, -0.0, float("inf"), 0.5e-9, 2e23, -0.3], dtype=np.float64)
    d_in = torch.from_numpy(xs).to(gpu)
    d_out = torch.empty_like(d_in)
    assert _capi.load().tbe_numfmt_device(d_in.data_ptr(), d_out.data_ptr(), xs.size, None) == 0
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    inside = (np.abs(xs) >= 1e-9) & (np.abs(xs) < 1e23)
    want = np.array([float("%.14g" % x) for x in xs[inside]])
    bad = np.flatnonzero(got[inside].view(np.uint64) != want.view(np.uint64))
    assert bad.size == 0, list(zip(xs[inside][bad[:5]], got[inside][bad[:5]], want[bad[:5]]))
    assert got[~inside][:3].tolist() == [0.0, 0.0, float("inf")]   # passed through
    assert inside.sum() > 500_000


@pytest.mark.parametrize("order", [OLDEST_FIRST, NEWEST_FIRST])
def test_zero_permit_waits_queue(engine_lib, gpu, order):
    """WaitAsync(0) while AvailableTokens is 0 queues with Count 0 (A:127-181), holds no
    queue permits, completes at the next drain that reaches it (A:474), is evicted from the
    head like any registration (A:145-156) and can be canceled; zero_wait_slots bounds
    them per key.  Hand-checked, and against the Python restatement."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    eng = ApproximateEngine(4, 2, 2, 10_000_000, 2, order, device=0, zero_wait_slots=2)
    cli = ApproxClient(2, 2, 10_000_000, 2, order, zero_slots=2)
    reqs = [(1, 2), (1, 0), (1, 0), (1, 0), (1, 1), (1, 1), (1, 2), (2, 0)]
    keys = np.array([k for k, _ in reqs], np.uint64)
    ps = np.array([p for _, p in reqs], np.int32)
    st, av, (cause, ids) = eng.acquire_batch(keys, ps, wait=True, id_base=100)
    exp = [cli.wait(k, p, 100 + i) for i, (k, p) in enumerate(reqs)]
    assert st.tolist() == [e[0] for e in exp]
    assert list(zip(cause.tolist(), ids.tolist())) == [(i, x) for i, e in enumerate(exp) for x in e[1]]
    # key 1: granted 2, two zero waits queue, the third finds no zero slot; p=1, p=1 queue
    # (qsum 2); p=2: OldestFirst fails, NewestFirst evicts the head run (zeros included)
    # until 2 permits fit; key 2 has tokens: a zero wait is granted at once
    if order == OLDEST_FIRST:
        assert st.tolist() == [1, 2, 2, 0, 2, 2, 0, 1]
    else:
        assert st.tolist() == [1, 2, 2, 0, 2, 2, 2, 1] and ids.tolist() == [101, 102, 104, 105]
    assert [q for q in eng.queue_of(1)] == [(e.request_id, e.permits) for e in cli.st(1).queue]
    # a cancel of a queued zero wait (OldestFirst only has one left to cancel here)
    if order == OLDEST_FIRST:
        assert eng.cancel(np.array([1], np.uint64), np.array([102], np.int64)).tolist() == [1]
        assert cli.cancel(1, 102)
    counts = torch.zeros(4, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()
    tbl = ApproxGlobalTable(cli.decay_rate)
    ts = S_US
    for epoch in range(3):
        ts += 1_000_000
        eng.collect(counts)
        log = eng.sync(counts, 1, 0, ts, 0)
        exp_log = approx_refresh_all([cli], tbl, ts, 0, range(4))[0]
        assert list(zip(log[0].tolist(), log[1].tolist())) == exp_log
        for key in range(4):
            lo, gl, est, a, q = eng.local_state(key)
            s = cli.st(key)
            assert (lo, gl, est, a, q) == (s.local, s.global_, s.est, cli.available(s), len(s.queue))


def test_global_tier_snapshot_restore(engine_lib, gpu):
    """tbe_approx_export_state -> tbe_approx_import_state (the Redis hash {v, p, t} with
    its one-day TTL, A:265-268): a replica restored into a fresh engine continues the
    sync replay exactly like the original; absent rows of a snapshot (t = INT64_MIN) read
    back as the script's default {0, 0} and behave like never-synced keys."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine, TbeError
    ABS = np.iinfo(np.int64).min
    n_keys, half = 5000, 2500
    mk = lambda: ApproximateEngine(n_keys, 50, 10, 10_000_000, 0, 0, device=0)
    a = mk()
    rng = np.random.default_rng(8)
    counts = torch.zeros(n_keys, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()
    v0, p0, t0 = a.export_global()
    assert (t0 == ABS).all() and (v0 == 0).all() and (p0 == 0).all()
    ts = S_US
    for epoch in range(3):
        keys = rng.integers(0, n_keys, 20_000).astype(np.uint64)
        a.acquire_batch(keys, rng.integers(0, 4, keys.size).astype(np.int32), wait=False)
        ts += 700_000
        a.collect(counts)
        a.sync(counts, 1, 0, ts, 0)
    v, p, t = a.export_global()
    assert (t == ts).all() and (p > 0).any()          # every key syncs every epoch (A:412-508)
    b = mk()                                          # restored in two ranges
    b.import_global(v[:100], p[:100], t[:100])
    b.import_global(v[100:], p[100:], t[100:], first=100)
    for x, y in zip(b.export_global(), (v, p, t)):
        assert np.array_equal(x.view(np.uint64), y.view(np.uint64))
    c = mk()                                          # upper half absent in the snapshot
    t2 = t.copy()
    t2[half:] = ABS
    c.import_global(np.full(n_keys, 7.0), np.full(n_keys, 3.0), t2)
    c.import_global(v[:half], p[:half], t[:half])
    vc, pc, tc = c.export_global()
    assert (tc[half:] == ABS).all() and (vc[half:] == 0).all() and (pc[half:] == 0).all()
    d = mk()                                          # lower half restored, upper never synced
    d.import_global(v[:half], p[:half], t[:half])
    for epoch in range(2):
        cn = torch.from_numpy(rng.integers(0, 30, n_keys).astype(np.int32)).to(gpu)
        ts += 900_000
        for e in (a, b, c, d):
            e.sync(cn, 1, 0, ts, 0)
        for x, y in zip(a.export_global(), b.export_global()):
            assert np.array_equal(x.view(np.uint64), y.view(np.uint64))
        for x, y in zip(c.export_global(), d.export_global()):
            assert np.array_equal(x.view(np.uint64), y.view(np.uint64))
        for key in range(0, n_keys, 37):
            assert a.local_state(key)[1:3] == b.local_state(key)[1:3]
            assert c.local_state(key)[1:3] == d.local_state(key)[1:3]
    # past the one-day TTL every key is absent again: the next sync starts from {0, 0, now}
    day = 86_400 * 1_000_000
    zero = torch.zeros(n_keys, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()
    b.sync(zero, 1, 0, ts + day + 2_000, 0)
    vb, pb, _ = b.export_global()
    assert (pb == 0.0).all() and (vb == 0.0).all()
    with pytest.raises(TbeError):
        b.import_global(v[:10], p[:10], t[:10], first=n_keys - 5)


def test_client_view_survives_import_after_one_client_sync(engine_lib, gpu):
    """Round 6: after a one-client sync the engine derives the client view {global, est}
    (A:441-443) from the tier row when asked instead of writing it every sync.  Importing
    another tier replica afterwards must not change the view -- the reference's client keeps
    the values of its last sync until its next one -- and a multi-client sync writes it
    again.  Views against the oracle client at every step."""
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, limit, tokens, ticks = 400, 30, 10, 10_000_000
    eng = ApproximateEngine(n_keys, limit, tokens, ticks, 0, 0, device=0)
    client = ApproxClient(limit, tokens, ticks, 0, 0)
    table = ApproxGlobalTable(client.decay_rate)
    rng = np.random.default_rng(21)
    counts = torch.zeros(n_keys, dtype=torch.int32, device=gpu)
    ts = S_US

    def views():
        return [eng.local_state(k)[1:3] for k in range(0, n_keys, 7)]

    def expect():
        return [(client.st(k).global_, client.st(k).est) for k in range(0, n_keys, 7)]

    for epoch in range(3):
        keys = rng.integers(0, n_keys, 3000).astype(np.uint64)
        permits = rng.integers(0, 4, keys.size).astype(np.int32)
        eng.acquire_batch(keys, permits, wait=False)
        for k, p in zip(keys.tolist(), permits.tolist()):
            client.acquire(k, p)
        ts += 800_000
        eng.collect(counts)
        torch.cuda.synchronize()
        eng.sync(counts, 1, 0, ts, 0)
        approx_refresh_all([client], table, ts, 0, range(n_keys))
        assert views() == expect(), epoch
    before = views()
    v, p, t = eng.export_global()
    eng.import_global(np.zeros_like(v), np.full_like(p, 0.25), t)   # another replica's rows
    assert views() == before                                          # the view is the last sync's
    eng.import_global(v, p, t)
    two = torch.cat([counts, counts])
    torch.cuda.synchronize()
    eng.sync(two, 2, 1, ts + 800_000, 1000)                           # a multi-client sync writes it
    assert all(isinstance(x[1], float) for x in views())
