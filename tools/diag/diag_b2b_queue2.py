"""Diagnostic (round 5): the intermittent serial queue mismatch.  Re-creates the failing
sequence (a fused-tick engine, then another engine with host synchronisation between
batches); checks the device inputs against the host arrays after the run, and on a
mismatch in batch 0 replays batch 0 on a fresh engine from the same device tensors.
Not a test."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import cref  # checker only
from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate

S_US = 1_760_572_800 * 1_000_000
gpu = torch.device("cuda", 0)


def make(n_keys, n, nb, seed):
    rng = np.random.default_rng(seed)
    t, host, ins = S_US, [], []
    for b in range(nb):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        t += 1_000 + (int(rng.integers(0, 3_000_000)) if b % 2 else 0)
        host.append((keys, permits, ts, t))
        ins.append(tuple(torch.from_numpy(a).to(gpu) for a in (keys.view(np.int64), permits, ts)))
    return host, ins


def run(tag, sync_each, fused, n_keys=200_000, n=1 << 18, nb=4, seed=16):
    host, ins = make(n_keys, n, nb, seed)
    cap = n_keys * 4
    outs = [(torch.full((n,), 255, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu)) for _ in range(nb)]
    logs = [(torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
             torch.empty(cap, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)) for _ in range(nb)]
    torch.cuda.synchronize()
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 16, 0, device=0, pipeline=False)
    for b in range(nb):
        if fused:
            eng.wait_batch_tick_device(*ins[b], *outs[b], b * n, host[b][3], *logs[b])
        else:
            eng.wait_batch_device(*ins[b], *outs[b], id_base=b * n)
        if sync_each:
            eng.synchronize()
    eng.synchronize()
    torch.cuda.synchronize()
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), 16, 0)
    res, inputs_ok = [], True
    for b in range(nb):
        keys, permits, ts, tick = host[b]
        inputs_ok &= bool(np.array_equal(ins[b][0].cpu().numpy().view(np.uint64), keys) and
                          np.array_equal(ins[b][1].cpu().numpy(), permits) and np.array_equal(ins[b][2].cpu().numpy(), ts))
        st2, rem2, _, _ = ref.acquire_batch(keys, permits, ts, b * n)
        if fused:
            ref.refresh(tick)
        st = outs[b][0].cpu().numpy()
        rem = outs[b][1].cpu().numpy()
        res.append(int(np.count_nonzero((st != st2) | (rem != rem2))))
    eng.close()
    line = f"{tag}: sync={sync_each} fused={fused} mismatches {res} inputs intact {inputs_ok}"
    if res[0]:
        # batch 0 again on a fresh engine from the same device tensors
        e2 = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, 16, 0, device=0, pipeline=False)
        o2 = (torch.full((n,), 255, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu))
        torch.cuda.synchronize()
        e2.wait_batch_device(*ins[0], *o2, id_base=0)
        e2.synchronize()
        r2 = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), 16, 0)
        st2, rem2, _, _ = r2.acquire_batch(*host[0][:3], 0)
        bad2 = int(np.count_nonzero((o2[0].cpu().numpy() != st2) | (o2[1].cpu().numpy() != rem2)))
        same = bool(torch.equal(o2[0], outs[0][0]) and torch.equal(o2[1], outs[0][1]))
        line += f"; batch 0 replayed on a fresh engine: {bad2} mismatches, identical to the first run's output {same}"
        e2.close()
    print(line, flush=True)


if __name__ == "__main__":
    for rep in range(3):
        run(f"rep{rep} a", False, True)
        run(f"rep{rep} b", True, True)
        run(f"rep{rep} c", True, False)
        run(f"rep{rep} d", False, False)
