"""World-size-2 runs of the multi-GPU protocol (cluster.py) with the HIP engine deciding.

Two rank processes share the one GPU of the test box (each with its own engine and
directory on cuda:0) and exchange over gloo: RCCL refuses two ranks on one device, and
everything else -- route kernels, device directory, engine calls, the cluster layer's
exchanges -- is the code a multi-GPU node runs.  Expected results are the same serial
references as tests/test_dist_gloo.py (there the ranks' engines are the oracle):

* token-bucket routing: per step, rank 0's batch then rank 1's on one serial table
  (PTB:42: one key space shared by every client);
* queued waits routed to their owners, a third of them canceled through route_cancel,
  then a replenish tick on every rank (Q:67-134, Q:480-506, Q:237-271);
* approximate epochs, both exchange modes (A:412-508 with the sync script A:241-270):
  every rank a client (all-gather) and the node as one client (all-reduce).

Each protocol runs on the host path (numpy batches, host directory, host-buffer engine
calls) and on the device path (CUDA tensors end to end).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests import _dist_workers as W
from tests import test_dist_gloo as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(worker: str, out_dir, *args: str, timeout: int = 150):
    """Both ranks as child processes (never exec'd from this GPU-initialised process)."""
    port = _port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_dist_workers.py"), worker, str(r),
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


@pytest.mark.gpu
@pytest.mark.parametrize("path,map_kind", [("host", "hash"), ("device", "hash"), ("device", "balanced")])
def test_route_batch_two_hip_ranks(gpu, oracle_lib, tmp_path, path, map_kind):
    _run_ranks("tb_route_worker_hip", tmp_path, path, map_kind)
    G.check_tb_route([np.load(tmp_path / f"tb_{r}.npz") for r in range(WORLD)])


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["host", "device"])
def test_route_wait_and_cancel_two_hip_ranks(gpu, tmp_path, path):
    _run_ranks("q_route_worker_hip", tmp_path, path)
    res = [np.load(tmp_path / f"q_{r}.npz") for r in range(WORLD)]
    G.check_q_route(res)
    assert sum(int(r[f"hit{s}"].sum()) for r in res for s in range(W.Q_STEPS)) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["clients", "node"])
def test_approx_epoch_two_hip_ranks(gpu, tmp_path, mode):
    _run_ranks("ap_epoch_worker_hip", tmp_path, mode)
    G.check_approx([np.load(tmp_path / f"ap_{mode}_{r}.npz") for r in range(WORLD)], mode)
