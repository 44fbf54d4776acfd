#!/bin/bash
# round 5: benches with the timed engine free of stage events (stage times from replays)
set -o pipefail
mkdir -p gpurun_out
for w in queue approx zipf; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r05p_bench_$w.json 2> gpurun_out/r05p_bench_$w.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05p_bench_$w.json').read().strip().splitlines()[-1])
print('$w', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
