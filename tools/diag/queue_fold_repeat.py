"""Diagnostic (round 6): why config D's fold runs slower in the bench's
timed engine than in the replay engine created right after it.

Runs config D's schedule (1e8 keys, QueueLimit 16, 2^26-request batches, fused ticks; 5
warm-up + 20 timed batches) on several engines in a row, each created, used and destroyed
in turn, and prints the fold's mean ms per timed batch (HIP events around the fold,
TBE_FLAG_FOLD_TIMING) and tbe_create's wall time for each.  Variants:
  fresh    create, run at once
  settle   create, wait `--settle` seconds, run
The first engine of a process gets memory no earlier engine of the process has used; the
later ones reuse what the earlier ones freed.  Not a test: prints what it measures.
usage: python tools/diag/queue_fold_repeat.py [--settle 3] [--pattern ffsf]
(pattern: one letter per engine, f = fresh, s = settle)"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench_kinds import _gen  # noqa: E402
from distributedratelimiting.redis_amd import QueueingTokenBucketEngine, _capi  # noqa: E402

N_KEYS, N, WARM, STEPS, INTERVAL = 100_000_000, 1 << 26, 5, 20, 1_000


def run(lib, dev, bufs, settle):
    t0 = time.perf_counter()
    eng = QueueingTokenBucketEngine(N_KEYS, 4, 1, 10_000_000, 16, 0, device=dev.index, stage_timing="fold",
                                    max_batch=N)
    create_s = time.perf_counter() - t0
    if settle:
        time.sleep(settle)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    rem = torch.empty(N, dtype=torch.int32, device=dev)
    cap = N_KEYS * 4          # tbe_refresh_bound: min(QueueLimit, TokenLimit) grants per key
    lk = torch.empty(cap, dtype=torch.int64, device=dev)
    li = torch.empty(cap, dtype=torch.int64, device=dev)
    lr = torch.empty(cap, dtype=torch.int32, device=dev)
    cnt = torch.zeros(WARM + STEPS, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    for s in range(WARM + STEPS):
        if s == WARM:
            eng.synchronize()
            eng.stage_times()
        eng.wait_batch_tick_device(*bufs[s], st, rem, s * N, 1_760_000_000_000_000 + (s + 1) * INTERVAL,
                                   lk, li, lr, cnt[s:s + 1], stream=stream.cuda_stream)
    eng.synchronize()
    fold = eng.stage_times().get("fold", 0.0) / STEPS
    eng.close()
    del st, rem, lk, li, lr
    return create_s, fold


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settle", type=float, default=3.0)
    ap.add_argument("--pattern", default="ffsf")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _capi.load()
    bufs = [_gen(lib, 0x5EED000D, N_KEYS, s, N, INTERVAL, dev) for s in range(WARM + STEPS)]
    torch.cuda.synchronize()
    for i, kind in enumerate(a.pattern):
        settle = a.settle if kind == "s" else 0.0
        c, f = run(lib, dev, bufs, settle)
        print(f"engine {i}: {'settle %.1fs' % settle if settle else 'fresh'}  create {c * 1e3:.1f} ms  "
              f"fold {f:.4f} ms per timed batch", flush=True)


if __name__ == "__main__":
    main()
