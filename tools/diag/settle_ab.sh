#!/bin/bash
# Diagnostic (round 6): does device-memory work left by an earlier process slow the next
# bench?  A process allocates, writes and frees 60 GB; then a bench starts at once, or after
# --settle-s 3.  Configs B and D, two rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$(pwd)/gpurun_out
TAG=${TAG:-r06h}
churn() { timeout -k 10 60 python -c "import torch; x = torch.empty(60 << 30, dtype=torch.uint8, device='cuda'); x.fill_(1); torch.cuda.synchronize(); print('churn', x.numel() >> 30, 'GB')"; }
for i in 1 2; do
  for w in uniform queue; do
    for st in 0 3; do
      churn || exit $?
      timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --no-host-buffer --no-strdir --no-sparse --no-drain-variant --settle-s $st > $OUT/${TAG}_settle_${w}_${st}_$i.log 2>&1 || exit $?
      python3 -c "import json; d=json.loads([l for l in open('$OUT/${TAG}_settle_${w}_${st}_$i.log') if l.startswith('{')][0]); r=d['roofline']; print('$w settle $st round $i', d['ms_per_step'], 'fold', r['avg_launch_ms'], d['stage_ms_per_step'])"
    done
  done
done
