"""bench.py's workload table and its algorithmic-byte model,
checked without a GPU."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(argv):
    sys.path.insert(0, ROOT)
    import bench
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("workload,batch,interval,limit,tokens", [
    ("uniform", 1 << 26, 10_000, 10, 1),       # config B
    ("zipf", 1 << 26, 10_000, 10, 1),          # config C (per-GPU slice)
    ("queue", 1 << 26, 1_000, 4, 1),           # config D
    ("approx", 1 << 26, 10_000, 100, 10),      # config E
    ("testapp", 1_000_000, 2_000_000, 20, 10),  # config A
])
def test_workload_defaults(workload, batch, interval, limit, tokens):
    a = parse(["--workload", workload])
    assert (a.batch, a.interval_us, a.token_limit, a.tokens_per_period) == (batch, interval, limit, tokens)
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0


def test_explicit_flags_win():
    a = parse(["--workload", "testapp", "--batch", "4096", "--token-limit", "7"])
    assert (a.batch, a.token_limit) == (4096, 7)


def test_algorithmic_bytes_model():
    sys.path.insert(0, ROOT)
    import bench
    n, k = 1 << 26, 100_000_000
    fold4 = bench.algorithmic_bytes("fold", n, k, 2, True, None, 4)
    fold1 = bench.algorithmic_bytes("fold", n, k, 2, True, None, 1)
    assert fold4 - fold1 == 3 * n                      # reply width
    u = k * (1 - pow(2.718281828459045, -n / k))
    assert abs(fold1 - (n * 9 + u * 32)) < n            # records 8 + reply 1, rows 32 per key
    # the decision's own minimum is <= 48.3 B per request at config B
    assert (n * 25 + u * 32) / n < 48.4


def _bench(argv, env_extra=None, timeout=240):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_n_refuses_without_n_devices():
    """--gpus 2 outside torchrun launches 2 ranks only if 2 GPUs are visible; here (no
    GPU) it must exit non-zero instead of printing a one-rank line."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible")
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0 and not p.stdout.strip()
    assert "--gpus 2 but only" in p.stderr


def test_world_size_mismatch_refuses():
    p = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and not p.stdout.strip()
    assert "world size 2 != --gpus 1" in p.stderr


def test_gpus_n_spawns_n_ranks():
    """--share-device skips the device count, so the launcher starts torch.distributed.run
    with 2 ranks: both report in (then fail without a GPU, and the launcher's exit status
    is non-zero, with no line printed)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible: the spawned ranks would run the benchmark")
    p = _bench(["--gpus", "2", "--share-device", "--steps", "1", "--warmup", "0"])
    # (gloo's own connection messages may reach stdout; no JSON line may)
    assert p.returncode != 0 and not [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert "bench.py: rank 0 of 2" in p.stderr and "bench.py: rank 1 of 2" in p.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("workload", ["uniform", "zipf", "queue", "approx"])
def test_gpus_2_rehearsal_on_one_gpu(workload):
    """The multi-rank bench path as the driver launches it (--gpus 2 spawns two ranks),
    rehearsed on the one GPU of the test box: both ranks on cuda:0 over gloo, the HIP
    engine deciding on each, the device path's collectives staged through host memory.
    One JSON line, for two GPUs' worth of work, marked as a rehearsal."""
    argv = ["--gpus", "2", "--share-device", "--workload", workload, "--keys", "2000000",
            "--batch", str(1 << 20), "--steps", "2", "--warmup", "1", "--cpu-seconds", "0",
            "--no-host-buffer", "--no-strdir"]
    if workload == "queue":
        argv.append("--no-drain-variant")
    if workload == "zipf":   # config C's form: one global Zipf stream, hash-sharded to its owners
        argv[argv.index("--keys") + 1] = "3000000"
    p = _bench(argv, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 2
    assert "rehearsal" in json.dumps(d)
