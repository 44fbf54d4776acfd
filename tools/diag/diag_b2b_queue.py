"""Diagnostic (round 5): back-to-back queue batches on one engine, per-batch mismatch
statistics against the C restatement.  Not a test: prints what differs.
usage: python tools/diag_b2b_queue.py  (TBE_LIB selects the engine library)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import cref  # checker only
from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, fill_rate

S_US = 1_760_572_800 * 1_000_000


def run(pipeline, sync_each, mode="fused", order=0, qlimit=16, n_keys=200_000, n=1 << 18, nb=4, seed=16):
    gpu = torch.device("cuda", 0)
    rng = np.random.default_rng(seed)
    eng = QueueingTokenBucketEngine(n_keys, 4, 1, 10_000_000, qlimit, order, device=0, pipeline=pipeline)
    ref = cref.CQueueingTokenBucket(n_keys, 4, fill_rate(1, 10_000_000), qlimit, order)
    cap = n_keys * min(max(qlimit, 1), 4)
    t, host, ins, outs, logs = S_US, [], [], [], []
    for b in range(nb):
        keys = rng.integers(0, n_keys, n).astype(np.uint64)
        permits = rng.choice([0, 1, 1, 1, 2, 3], n).astype(np.int32)
        ts = (t + np.sort(rng.integers(0, 1_000, n))).astype(np.int64)
        t += 1_000 + (int(rng.integers(0, 3_000_000)) if b % 2 else 0)
        host.append((keys, permits, ts, t))
        ins.append(tuple(torch.from_numpy(a).to(gpu) for a in (keys.view(np.int64), permits, ts)))
        outs.append((torch.full((n,), 255, dtype=torch.uint8, device=gpu), torch.empty(n, dtype=torch.int32, device=gpu)))
        logs.append((torch.empty(cap, dtype=torch.int64, device=gpu), torch.empty(cap, dtype=torch.int64, device=gpu),
                     torch.empty(cap, dtype=torch.int32, device=gpu), torch.zeros(1, dtype=torch.int32, device=gpu)))
    torch.cuda.synchronize()
    for b in range(nb):
        if mode == "fused":
            eng.wait_batch_tick_device(*ins[b], *outs[b], b * n, host[b][3], *logs[b])
        else:
            eng.wait_batch_device(*ins[b], *outs[b], id_base=b * n)
            if mode == "unfused":
                eng.refresh_device(host[b][3], *logs[b])
        if sync_each:
            eng.synchronize()
    eng.synchronize()
    torch.cuda.synchronize()
    res = []
    for b in range(nb):
        keys, permits, ts, tick = host[b]
        st2, rem2, _, _ = ref.acquire_batch(keys, permits, ts, b * n)
        if mode != "waitonly":
            ref.refresh(tick)
        st = outs[b][0].cpu().numpy()
        rem = outs[b][1].cpu().numpy()
        bad = np.flatnonzero((st != st2) | (rem != rem2))
        res.append(int(bad.size))
        if bad.size and len([r for r in res if r]) == 1:
            j = bad[:6]
            bk = keys[bad] >> np.uint64(8)
            print(f"    first bad batch {b}: idx {j.tolist()} gpu st {st[j].tolist()} rem {rem[j].tolist()} ref st {st2[j].tolist()} rem {rem2[j].tolist()}; "
                  f"buckets {np.unique(bk).size}, st==255: {(st[bad] == 255).sum()}", flush=True)
    print(f"lib={os.path.basename(os.environ.get('TBE_LIB', 'libtbe.so'))} pipeline={eng.layout()['pipeline']} "
          f"sync_each={sync_each} mode={mode} keys={n_keys} n={n}: mismatches per batch {res}", flush=True)
    eng.close()


if __name__ == "__main__":
    for args in [(False, False), (False, True), (False, True, "unfused"), (False, True, "waitonly"),
                 (False, False, "waitonly"), (False, True), (False, False)]:
        run(*args)
    run(False, True, "fused", 0, 16, 5000, 60000)
    run(False, True, "fused", 0, 16, 1_000_000, 1 << 20)
    if "head" not in os.environ.get("TBE_LIB", ""):
        run(True, False)
        run(True, True)
