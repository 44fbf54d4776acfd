#!/bin/bash
# One gpurun call for the edit -> measure loop: GPU parity tests, the config-B bench and
# the config-C (Zipf) bench.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest rc=$?"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --steps "${STEPS:-5}" --warmup 3 --cpu-seconds "${CPU_S:-0}" \
    > "$OUT/bench_u.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/bench_u.log"; exit 1; }
timeout -k 10 400 python -u bench.py --workload zipf --steps "${STEPS:-5}" --warmup 3 --cpu-seconds "${CPU_S:-0}" \
    > "$OUT/bench_z.log" 2>&1 || { echo "zipf bench rc=$?"; tail -5 "$OUT/bench_z.log"; exit 1; }
echo cycle-done
