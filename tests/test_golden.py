"""The CPU restatements against golden vectors recorded by executing the reference's
own Lua scripts (tests/golden/make_golden.py + oracle/lua_replay.py)."""
import glob
import os

import numpy as np
import pytest

from oracle import cref
from oracle.semantics import (ApproxGlobalTable, TokenBucketConfig, TokenBucketTable,
                              instance_count_estimate, new_t_of)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TB_CASES = sorted(glob.glob(os.path.join(GOLDEN, "tb_*.npz")))
APPROX_CASES = sorted(glob.glob(os.path.join(GOLDEN, "approx_*.npz")))


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_fixtures_present():
    assert len(TB_CASES) >= 7 and len(APPROX_CASES) >= 3


@pytest.mark.parametrize("path", TB_CASES, ids=os.path.basename)
def test_python_oracle_matches_golden(path):
    g = load(path)
    tb = TokenBucketTable(TokenBucketConfig(int(g["token_limit"]), float(g["fill_rate"])))
    granted, remaining = tb.acquire_batch(g["keys"], g["permits"], g["ts_us"])
    assert np.array_equal(np.array(granted, np.uint8), g["granted"])
    assert np.array_equal(np.array(remaining, np.int32), g["remaining"])
    for k in range(int(g["n_keys"])):
        st = tb.query(k)
        if g["present"][k]:
            assert st is not None and st[0] == g["v"][k] and st[1] == g["t"][k]
        else:
            assert st is None


@pytest.mark.parametrize("path", TB_CASES, ids=os.path.basename)
def test_c_oracle_matches_golden(path, oracle_lib):
    g = load(path)
    n_keys = int(g["n_keys"])
    c = cref.CTokenBucket(n_keys, int(g["token_limit"]), float(g["fill_rate"]))
    granted, remaining = c.acquire_batch(g["keys"], g["permits"], g["ts_us"])
    assert np.array_equal(granted, g["granted"]) and np.array_equal(remaining, g["remaining"])
    v, t_us = c.export_state()
    absent = np.iinfo(np.int64).min
    for k in range(n_keys):
        if g["present"][k]:
            assert v[k] == g["v"][k] and new_t_of(int(t_us[k])) == g["t"][k]
        else:
            assert t_us[k] == absent


@pytest.mark.parametrize("path", APPROX_CASES, ids=os.path.basename)
def test_approx_sync_matches_golden(path):
    g = load(path)
    tbl = ApproxGlobalTable(float(g["decay_rate"]))
    for i in range(len(g["counts"])):
        score, period, s = tbl.sync("approx:default", int(g["counts"][i]), int(g["ts_us"][i]))
        assert score == g["global_score"][i]
        assert s == str(g["period_str"][i]) and period == g["period"][i]
    st = tbl.state["approx:default"]
    assert (st.v, st.p, new_t_of(st.t_us)) == (g["final_v"], g["final_p"], g["final_t"])


def test_instance_count_estimate_warmup():
    # one client, refresh every P = 1 s: est after each sync = inf, 5, 3, 2, 2, 1, 1, 1
    tbl = ApproxGlobalTable(10.0)
    t0 = 1_760_572_800 * 1_000_000
    est = []
    for i in range(8):
        _, period, _ = tbl.sync("k", 0, t0 + i * 1_000_000)
        est.append(instance_count_estimate(1.0, period))
    assert est == [float("inf"), 5.0, 3.0, 2.0, 2.0, 1.0, 1.0, 1.0]
