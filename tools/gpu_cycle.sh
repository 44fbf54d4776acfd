#!/bin/bash
# One gpurun call for the edit -> measure loop: GPU parity tests, the config-B bench and
# the config-C (Zipf) bench, each also with AB_FLAGS (e.g. AB_FLAGS=--no-pipeline) when
# set.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest rc=$?"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run_bench() {   # name, extra args...
    local name=$1
    shift
    timeout -k 10 400 python -u bench.py --steps "${STEPS:-5}" --warmup 3 --cpu-seconds "${CPU_S:-0}" "$@" \
        > "$OUT/bench_$name.log" 2>&1 || { echo "bench $name rc=$?"; tail -5 "$OUT/bench_$name.log"; return 1; }
    tail -1 "$OUT/bench_$name.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
}
run_bench u || exit 1
if [ -n "${AB_FLAGS:-}" ]; then run_bench u_ab $AB_FLAGS || exit 1; fi
run_bench z --workload zipf || exit 1
if [ -n "${AB_FLAGS:-}" ]; then run_bench z_ab --workload zipf $AB_FLAGS || exit 1; fi
echo cycle-done
