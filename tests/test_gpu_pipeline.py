"""Back-to-back device batches through the pipelined token-bucket engine.

A pipelined engine keeps two batch workspaces and runs a batch's partition passes on one
HIP stream and its fold, hot runs and unscatter on another, so batch b+1 is partitioned
while batch b is folded.  Every batch's replies and the final table must
still equal the C restatement's (oracle/tb_ref.c), bit for bit:

- enqueued with no stream (inputs complete at the call, replies complete at
  tbe_synchronize), uniform and Zipf traffic (hot sets rotate across batches);
- enqueued on a caller stream that regenerates the inputs in place after every call (the
  engine waits on that stream for the inputs and makes it wait for the replies);
- with an invalid batch in the middle of the sequence (skipped, reported by
  tbe_synchronize, later batches applied).
"""
import ctypes

import numpy as np
import pytest

from oracle import cref, trace

pytestmark = pytest.mark.gpu

ABSENT = np.iinfo(np.int64).min
SEED = 0x5EED0A0B


def _lib():
    from distributedratelimiting.redis_amd import _capi
    lib = _capi.load()
    lib.tbe_gen_batch_device.restype = ctypes.c_int
    lib.tbe_gen_batch_device.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_int32] * 2 + \
        [ctypes.c_int64] * 2 + [ctypes.c_void_p] * 4
    return lib


def _gen(lib, n_keys, b, n, bufs, stream=None):
    dk, dp, dt = bufs
    rc = lib.tbe_gen_batch_device(SEED, n_keys, b * n, n, 1, 4, trace.T0_US + b * 10_000, 10_000,
                                  dk.data_ptr(), dp.data_ptr(), dt.data_ptr(), stream)
    assert rc == 0


def _inputs(torch, gpu, n):
    return (torch.empty(n, dtype=torch.int64, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu),
            torch.empty(n, dtype=torch.int64, device=gpu))


def _outputs(torch, gpu, n):
    return torch.empty(n, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu)


def _same_state(eng, ref):
    v, t = eng.export_state()
    v_ref, t_ref = ref.export_state()
    assert np.array_equal(t, t_ref), f"t mismatch at {np.flatnonzero(t != t_ref)[:10]}"
    touched = t_ref != ABSENT
    bad = np.flatnonzero(v[touched].view(np.uint64) != v_ref[touched].view(np.uint64))
    assert bad.size == 0, f"v mismatch at {np.flatnonzero(touched)[bad[:10]]}"


def _check_batch(b, out, g_ref, r_ref):
    g = out[0].cpu().numpy()
    r = out[1].cpu().numpy()
    bad = np.flatnonzero((g != g_ref) | (r != r_ref))
    assert bad.size == 0, f"batch {b}: {bad.size} mismatches, first at {bad[:5]}"


@pytest.mark.parametrize("pipeline", [True, False], ids=["pipelined", "serial"])
def test_back_to_back_device_batches(engine_lib, gpu, pipeline):
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    lib = _lib()
    n_keys, n, nb = 1_000_000, 1 << 18, 6
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0, pipeline=pipeline)
    assert eng.layout()["pipeline"] == pipeline
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    ins = [_inputs(torch, gpu, n) for _ in range(nb)]
    outs = [_outputs(torch, gpu, n) for _ in range(nb)]
    for b in range(nb):
        _gen(lib, n_keys, b, n, ins[b])
    torch.cuda.synchronize()
    for b in range(nb):
        eng.acquire_batch_device(*ins[b], *outs[b])
    eng.synchronize()
    for b in range(nb):
        k, p, t = trace.make_batch(SEED, n_keys, b, n, 10_000, 1, 4)
        _check_batch(b, outs[b], *ref.acquire_batch(k, p, t))
    _same_state(eng, ref)


def test_back_to_back_zipf_hot_rotation(engine_lib, gpu):
    """Zipf(1.1): the hot set nominated by batch b partitions batch b+2 while batch b+1 is
    partitioned during batch b's fold; replies and state stay exact."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate, workloads
    n_keys, n, nb = 1_000_000, 1 << 20, 6
    eng = TokenBucketEngine(n_keys, 20, 50, 10_000_000, device=0)
    lay = eng.layout()
    assert lay["pipeline"] and lay["hot"]
    ref = cref.CTokenBucket(n_keys, 20, fill_rate(50, 10_000_000))
    zs = workloads.ZipfSampler(n_keys, 1.1)
    rng = np.random.default_rng(8)
    host, ins, outs = [], [], []
    for b in range(nb):
        k = workloads.zipf_keys(SEED, n_keys, b * n, n, sampler=zs)
        p = np.where(rng.random(n) < 0.95, 1, rng.integers(0, 23, n)).astype(np.int32)
        t = workloads.batch_timestamps(b, n, 10_000, trace.T0_US)
        host.append((k, p, t))
        ins.append((torch.from_numpy(k.view(np.int64)).to(gpu), torch.from_numpy(p).to(gpu),
                    torch.from_numpy(t).to(gpu)))
        outs.append(_outputs(torch, gpu, n))
    torch.cuda.synchronize()
    for b in range(nb):
        eng.acquire_batch_device(*ins[b], *outs[b])
    eng.synchronize()
    for b in range(nb):
        _check_batch(b, outs[b], *ref.acquire_batch(*host[b]))
    _same_state(eng, ref)


def test_caller_stream_reuses_inputs(engine_lib, gpu):
    """One caller stream regenerates the same input buffers after every call and copies
    the replies out; only that stream is synchronised before the replies are read."""
    import torch
    from distributedratelimiting.redis_amd import TokenBucketEngine, fill_rate
    lib = _lib()
    n_keys, n, nb = 300_000, 1 << 17, 5
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0)
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    s = torch.cuda.Stream(device=gpu)
    bufs = _inputs(torch, gpu, n)
    out = _outputs(torch, gpu, n)
    copies = []
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for b in range(nb):
            _gen(lib, n_keys, b, n, bufs, stream=s.cuda_stream)
            eng.acquire_batch_device(*bufs, *out, stream=s.cuda_stream)
            copies.append((out[0].clone(), out[1].clone()))
    s.synchronize()
    for b in range(nb):
        k, p, t = trace.make_batch(SEED, n_keys, b, n, 10_000, 1, 4)
        _check_batch(b, copies[b], *ref.acquire_batch(k, p, t))
    eng.synchronize()
    _same_state(eng, ref)


def test_invalid_batch_in_pipeline(engine_lib, gpu):
    import torch
    from distributedratelimiting.redis_amd import TbeError, TokenBucketEngine, fill_rate
    lib = _lib()
    n_keys, n, nb, bad_b = 200_000, 1 << 16, 4, 2
    eng = TokenBucketEngine(n_keys, 10, 1, 10_000_000, device=0)
    ref = cref.CTokenBucket(n_keys, 10, fill_rate(1, 10_000_000))
    ins = [_inputs(torch, gpu, n) for _ in range(nb)]
    outs = [_outputs(torch, gpu, n) for _ in range(nb)]
    for b in range(nb):
        _gen(lib, n_keys, b, n, ins[b])
    ins[bad_b][0][777] = n_keys          # key out of range: the whole batch is skipped
    torch.cuda.synchronize()
    for b in range(nb):
        eng.acquire_batch_device(*ins[b], *outs[b])
    with pytest.raises(TbeError) as ei:
        eng.synchronize()
    assert ei.value.status == 1
    eng.synchronize()                    # the sticky flag was cleared
    for b in range(nb):
        if b == bad_b:
            continue
        k, p, t = trace.make_batch(SEED, n_keys, b, n, 10_000, 1, 4)
        _check_batch(b, outs[b], *ref.acquire_batch(k, p, t))
    _same_state(eng, ref)
