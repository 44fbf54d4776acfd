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


@pytest.mark.parametrize("n_clients,order,qlimit,wait", [(1, OLDEST_FIRST, 8, True), (3, NEWEST_FIRST, 4, True),
                                                         (8, OLDEST_FIRST, 16, True), (2, OLDEST_FIRST, 0, False)])
def test_clients_epochs(engine_lib, gpu, n_clients, order, qlimit, wait):
    import torch
    from distributedratelimiting.redis_amd import ApproximateEngine
    n_keys, n, limit, tokens, ticks = 300, 4000, 20, 10, 10_000_000
    rng = np.random.default_rng(n_clients * 100 + order * 10 + qlimit)
    engines = [ApproximateEngine(n_keys, limit, tokens, ticks, qlimit, order, device=0) for _ in range(n_clients)]
    clients = [ApproxClient(limit, tokens, ticks, qlimit, order) for _ in range(n_clients)]
    table = ApproxGlobalTable(clients[0].decay_rate)
    counts = [torch.zeros(n_keys, dtype=torch.int32, device=gpu) for _ in range(n_clients)]
    rid = 0
    for epoch in range(6):
        for r in range(n_clients):
            keys = rng.integers(0, n_keys, n).astype(np.uint64)
            permits = rng.choice([0, 1, 1, 2, 3, 25], n).astype(np.int32)
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
        logs = [engines[r].sync(allc, n_clients, r, ts, stagger) for r in range(n_clients)]
        exp_logs = approx_refresh_all(clients, table, ts, stagger, range(n_keys))
        for r in range(n_clients):
            k, i, _ = logs[r]
            assert list(zip(k.tolist(), i.tolist())) == exp_logs[r]
        for r in range(n_clients):
            for key in range(0, n_keys, 7):
                lo, gl, est, av, q = engines[r].local_state(key)
                s = clients[r].st(key)
                assert (lo, gl, est, av, q) == (s.local, s.global_, s.est, clients[r].available(s), len(s.queue))
