#!/bin/bash
# One gpurun call: every GPU test, then the bench lines of configs B, C, D, E and a
# rocprofv3 kernel trace of each (B with --no-pipeline so kernel durations match the
# bench's serial-replay roofline).  Stops at the first step that faults or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
if [ "${TESTS:-1}" = "1" ]; then
    step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
fi
for W in ${WORKLOADS:-uniform zipf queue approx}; do
    step bench_$W 420 python -u bench.py --workload $W --steps ${STEPS:-10} --warmup 3 --cpu-seconds ${CPUS:-10}
done
if [ "${PROFILE:-1}" = "1" ]; then
    cd /tmp && export TMPDIR=/tmp
    for W in ${WORKLOADS:-uniform zipf queue approx}; do
        step rocprof_$W 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$W" -o run -- \
            python3 "$ROOT/bench.py" --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer
    done
    cd "$ROOT"
fi
echo done
