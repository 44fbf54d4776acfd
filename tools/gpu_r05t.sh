#!/bin/bash
# round 5: the queue and approximate benches with fold-only events in the timed engine,
# and a kernel trace of the queue bench to check the fold time against rocprof
set -o pipefail
mkdir -p gpurun_out
for w in queue approx; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r05t_bench_$w.json 2> gpurun_out/r05t_bench_$w.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05t_bench_$w.json').read().strip().splitlines()[-1])
print('$w', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stage_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05t_prof_queue" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload queue --steps 20 --warmup 5 --cpu-seconds 0 --no-drain-variant > "$GRAFT_REPO_ROOT/gpurun_out/r05t_prof_queue.log" 2>&1 || exit $?
echo prof-done
