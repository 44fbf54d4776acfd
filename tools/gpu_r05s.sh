#!/bin/bash
# round 5: config D's timed engine against its stage replay -- allocation-order A/B
set -o pipefail
mkdir -p gpurun_out
for o in base dummy bufs base; do
  TBE_BENCH_QUEUE_ORDER=$o timeout -k 10 300 python -u bench.py --workload queue --steps 20 --warmup 5 --cpu-seconds 0 --no-drain-variant > gpurun_out/r05s_q_$o.json 2> gpurun_out/r05s_q_$o.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05s_q_$o.json').read().strip().splitlines()[-1])
print('$o', d['ms_per_step'], d['stage_ms_per_step']['fold'])"
done
