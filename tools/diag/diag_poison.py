"""Diagnostic (round 5): does the queue fold read memory it never wrote?  Device memory is
filled with a pattern and handed back to the driver before each engine is created, so an
uninitialised read gives the same wrong answer every time; then the layout switches
(fold records, digit stream, packing, narrow replies) localise it.  Not a test."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import cref  # checker only
from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, TokenBucketEngine, fill_rate

S_US = 1_760_572_800 * 1_000_000


def poison(byte):
    x = torch.full((3 << 30,), byte, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()


def run(kind="queue", pb=None, sync_each=True, n_keys=200_000, n=1 << 18, nb=3, seed=16, **kw):
    gpu = torch.device("cuda", 0)
    if pb is not None:
        poison(pb)
    rng = np.random.default_rng(seed)
    if kind == "queue":
        eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 16, 0, device=0, pipeline=False, **kw)
        ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), 16, 0)
    else:
        eng = TokenBucketEngine(n_keys, 4, 1, 10_000_000, device=0, pipeline=False, **kw)
        ref = cref.CTokenBucket(n_keys, 4, fill_rate(1, 10_000_000))
    t, host, ins, outs = S_US, [], [], []
    for b in range(nb):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        t += 1_000
        host.append((keys, permits, ts))
        ins.append(tuple(torch.from_numpy(a).to(gpu) for a in (keys.view(np.int64), permits, ts)))
        outs.append((torch.full((n,), 255, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu)))
    torch.cuda.synchronize()
    for b in range(nb):
        if kind == "queue":
            eng.wait_batch_device(*ins[b], *outs[b], id_base=b * n)
        else:
            eng.acquire_batch_device(*ins[b], *outs[b])
        if sync_each:
            eng.synchronize()
    eng.synchronize()
    res = []
    for b in range(nb):
        keys, permits, ts = host[b]
        if kind == "queue":
            st2, rem2, _, _ = ref.acquire_batch(keys, permits, ts, b * n)
        else:
            st2, rem2 = ref.acquire_batch(keys, permits, ts)
        st = outs[b][0].cpu().numpy()
        rem = outs[b][1].cpu().numpy()
        res.append(int(np.count_nonzero((st != st2) | (rem != rem2))))
    print(f"{kind} poison={pb} sync={sync_each} {kw} keys={n_keys} n={n}: {res} layout={eng.layout()}", flush=True)
    eng.close()


if __name__ == "__main__":
    for pb in (None, 0x5A, 0x00, 0xFF):
        run(pb=pb)
    for kw in ({"fold_records": False}, {"digit_stream": False}, {"narrow": False}, {"pack": False}):
        run(pb=0x5A, **kw)
    run(pb=0x5A, sync_each=False)
    run("tb", pb=0x5A)
    run(pb=0x5A, n_keys=1_000_000, n=1 << 20)
    run(pb=0x5A, n_keys=5000, n=60000)
