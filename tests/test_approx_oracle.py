"""The C restatement of the approximate limiter (oracle/tb_ref.c tba_*, the config-E checker
and CPU baseline) against the Python restatement (oracle/semantics.py ApproxClient +
ApproxGlobalTable, whose sync script is pinned by the Lua-replay golden vectors): every
status, AvailableTokens, eviction, drain-log entry and the per-key state, bit for bit."""
import numpy as np
import pytest

from oracle import cref
from oracle.semantics import (AP_FAILED, AP_GRANTED, AP_QUEUED, NEWEST_FIRST, OLDEST_FIRST, ApproxClient,
                              ApproxGlobalTable, approx_refresh_all)

S_US = 1_760_572_800 * 1_000_000


@pytest.mark.parametrize("n_clients,order,qlimit,wait,zero", [
    (1, OLDEST_FIRST, 8, True, 4), (3, NEWEST_FIRST, 4, True, 2), (4, OLDEST_FIRST, 16, True, 0),
    (2, OLDEST_FIRST, 0, False, 4), (2, NEWEST_FIRST, 3, True, 5)])
def test_c_vs_python(oracle_lib, n_clients, order, qlimit, wait, zero):
    n_keys, n, limit, tokens, ticks = 200, 3000, 20, 10, 10_000_000
    rng = np.random.default_rng(n_clients * 31 + qlimit + zero)
    cs = [cref.CApprox(n_keys, limit, tokens, ticks, qlimit, order, zero) for _ in range(n_clients)]
    ps = [ApproxClient(limit, tokens, ticks, qlimit, order, zero_slots=zero) for _ in range(n_clients)]
    table = ApproxGlobalTable(ps[0].decay_rate)
    rid = 0
    for epoch in range(6):
        for r in range(n_clients):
            keys = rng.integers(0, n_keys, n).astype(np.uint64)
            permits = rng.choice([0, 0, 1, 1, 2, 3, 25], n).astype(np.int32)
            st, av, cause, ids = cs[r].acquire_batch(keys, permits, wait=wait, id_base=rid,
                                                     threads=1 + (epoch % 3))
            exp = []
            for i, (k, p) in enumerate(zip(keys.tolist(), permits.tolist())):
                c = ps[r]
                status, ev = c.wait(k, p, rid + i) if wait else (c.acquire(k, p), [])
                exp.append((status, -1 if status == 3 else c.available(c.st(k)), ev))
            assert st.tolist() == [x[0] for x in exp]
            assert av.tolist() == [x[1] for x in exp]
            assert list(zip(cause.tolist(), ids.tolist())) == [(i, x) for i, e in enumerate(exp) for x in e[2]]
            rid += n
        ts = S_US + epoch * 1_000_000 + int(rng.integers(0, 300_000))
        stagger = 1_000_000 // n_clients
        allc = np.concatenate([c.collect() for c in cs])
        logs = [cs[r].sync(allc, n_clients, r, ts, stagger, threads=1 + (r % 4)) for r in range(n_clients)]
        exp_logs = approx_refresh_all(ps, table, ts, stagger, range(n_keys))
        for r in range(n_clients):
            k, i, a = logs[r]
            assert list(zip(k.tolist(), i.tolist())) == exp_logs[r]
            x = cs[r].export()
            for key in range(n_keys):
                s = ps[r].st(key)
                assert (x["local"][key], x["global"][key], x["est"][key], x["available"][key],
                        x["queued"][key]) == (s.local, s.global_, s.est, ps[r].available(s), len(s.queue))
                assert cs[r].queue_of(key) == [(e.request_id, e.permits) for e in s.queue]
        for key in range(n_keys):
            st = table.state.get(f"approx:{key}")
            x = cs[0].export()
            assert (x["v"][key], x["p"][key], x["t_us"][key]) == (st.v, st.p, st.t_us)


def test_zero_permit_waits_python():
    """A:127-181 + A:474: zero-permit waits queue with Count 0 while throttled, take no
    queue permits, complete at the next drain that reaches them; zero_slots bounds them."""
    c = ApproxClient(2, 2, 10_000_000, 2, OLDEST_FIRST, zero_slots=2)
    tbl = ApproxGlobalTable(c.decay_rate)
    out = [c.wait(7, p, i)[0] for i, p in enumerate([2, 0, 1, 0, 0])]
    assert out == [AP_GRANTED, AP_QUEUED, AP_QUEUED, AP_QUEUED, AP_FAILED]
    assert [(e.request_id, e.permits) for e in c.st(7).queue] == [(1, 0), (2, 1), (3, 0)]
    assert c.st(7).qcount == 1                       # zero waits hold no queue permits
    # first sync: global 2, est inf -> cap 0: only the zero wait at the head completes
    log = approx_refresh_all([c], tbl, S_US, 0, [7])[0]
    assert log == [(7, 1)]
    # the p=1 entry blocks the zero wait behind it (queue order) ...
    assert [e.request_id for e in c.st(7).queue] == [2, 3]
    # ... until one period later: local was swapped to 0, v decays 2 -> 0 (rate 2/s), est
    # 5, cap ceil(2 / 5) = 1: the p=1 entry completes, then the zero wait behind it
    log = approx_refresh_all([c], tbl, S_US + 1_000_000, 0, [7])[0]
    assert log == [(7, 2), (7, 3)] and c.st(7).queue == []
