"""The sharded path at sizes that exercise it: two HIP-engine ranks
on the box's GPU over gloo (RCCL refuses two ranks on one device; everything else is the
code an 8-GPU node runs), every reply, drain log, eviction, cancel hit and owned table row
against one serial C restatement of the global stream (tests/_dist_large.py).

* config C's form: one global Zipf(1.1) stream over 2^24 keys, 2^22 requests per rank per
  step, 4 steps -- the route kernels' owner partition runs over 1024 tiles per step, the
  owners' directories assign millions of ids, the engine runs two LSD passes over ~4000
  buckets, and hot-key runs (keys with >= 2048 requests at their owner) are active from
  the third batch; routed before the steps (bench.py --route pre) and inside every step
  (cluster.route_batch), and with a balanced owner map (cluster.balanced_owner_map from
  the all-reduced virtual-node loads of step 0).  Config B's uniform stream at the same
  size, routed before.
* queued waits over 2^17 keys, 2^18 per rank per step, routed cancels, replenish ticks;
  OldestFirst and NewestFirst (evictions compared too).  Anchors: PTB:42, Q:67-134,
  Q:480-506, Q:237-271.
* approximate clients over 2^17 shared keys with queued waits and cancels, both exchange
  modes (A:116-214, A:439 with A:241-270).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2
pytestmark = pytest.mark.gpu


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(worker: str, out_dir, *args, timeout: int = 240):
    """Both ranks as child processes (never exec'd from this GPU-initialised process)."""
    port = _port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_dist_large.py"), worker, str(r),
                               str(WORLD), str(port), str(out_dir), *args],
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(WORLD)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} of {worker} failed ({p.returncode}):\n{o[-4000:]}"


def _load(tmp_path, name):
    return [dict(np.load(tmp_path / f"{name}_{r}.npz")) for r in range(WORLD)]


@pytest.mark.parametrize("keyspace,route_mode,map_kind", [
    ("zipf", "pre", "hash"), ("zipf", "step", "hash"), ("zipf", "pre", "balanced"), ("uniform", "pre", "hash")])
def test_sharded_token_bucket_full_stream(engine_lib, oracle_lib, gpu, tmp_path, keyspace, route_mode, map_kind):
    _run_ranks("tb_large_worker", tmp_path, keyspace, route_mode, map_kind)
    res = _load(tmp_path, f"tbl_{keyspace}_{route_mode}_{map_kind}")
    n, steps = int(res[0]["n"]), int(res[0]["steps"])
    for r, x in enumerate(res):
        assert x["mism_g"].sum() == 0 and x["mism_r"].sum() == 0, (r, x["mism_g"], x["mism_r"])
        assert int(x["tab_t"]) == 0 and int(x["tab_v"]) == 0, (r, x["tab_t"], x["tab_v"])
        assert int(x["stray"]) == 0 and int(x["ids_in_range"]) == 1
        assert int(x["ids_unique"]) == int(x["n_owned"])      # the directory's ids are distinct
        assert int(x["passes"]) == 2
        assert np.array_equal(x["recv"], x["load"])           # each owner received exactly its keys
    # every request of the global stream was decided by exactly one owner
    assert np.array_equal(sum(x["load"] for x in res), np.full(steps, WORLD * n))
    if keyspace == "zipf":
        # hot keys at their owner (>= 2048 requests in a batch) took hot-key runs
        assert max(int(x["max_mult"].max()) for x in res) >= 100_000
        assert max(float(x["hot_ms"]) for x in res) > 0.0
        loads = np.array([x["load"] for x in res], dtype=np.float64)
        if map_kind == "hash":
            assert (loads.max(0) / loads.mean(0)).max() > 1.02  # the hot keys load their owner unevenly
        else:
            assert (loads.max(0) / loads.mean(0)).max() < 1.02  # the balanced owner map evens them out


@pytest.mark.parametrize("order", [0, 1])
def test_sharded_queue_routed_cancel_and_tick(engine_lib, oracle_lib, gpu, tmp_path, order):
    _run_ranks("q_large_worker", tmp_path, str(order))
    res = _load(tmp_path, f"ql_{order}")
    for r, x in enumerate(res):
        for k in ("mism_st", "mism_rem", "mism_hit", "mism_log"):
            assert x[k].sum() == 0, (r, k, x[k])
        if order == 1:
            assert x["mism_ev"].sum() == 0, (r, x["mism_ev"])
        assert int(x["tab"]) == 0 and int(x["queues"]) == 0, (r, x["tab"], x["queues"])
    assert sum(int(x["queued"].sum()) for x in res) > 10_000
    assert sum(int(x["hits"].sum()) for x in res) > 1_000
    assert sum(int(x["log_len"].sum()) for x in res) > 0


@pytest.mark.parametrize("mode,order", [("clients", 0), ("node", 0), ("clients", 1)])
def test_sharded_approximate_epochs(engine_lib, oracle_lib, gpu, tmp_path, mode, order):
    _run_ranks("ap_large_worker", tmp_path, mode, str(order))
    res = _load(tmp_path, f"apl_{mode}_{order}")
    for r, x in enumerate(res):
        for k in ("mism_st", "mism_av", "mism_ev", "mism_hit", "mism_log"):
            assert x[k].sum() == 0, (r, k, x[k])
        assert int(x["glob"]) == 0 and int(x["loc"]) == 0, (r, x["glob"], x["loc"])
    assert sum(int(x["queued"].sum()) for x in res) > 10_000
    assert sum(int(x["hits"].sum()) for x in res) > 1_000
    assert sum(int(x["log_len"].sum()) for x in res) > 0
