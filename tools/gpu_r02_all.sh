#!/bin/bash
# Round-2 measurement of every workload: bench line (N=1), rocprofv3 kernel stats
# (--no-pipeline and the bench's own step counts, so kernel durations match the serial
# replay the roofline uses) and the
# HBM PMC passes (tools/pmc_all.sh).  Each GPU step has its own time limit; a failure
# ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r02}
for W in ${WORKLOADS:-uniform zipf queue approx}; do
    timeout -k 10 420 python -u bench.py --workload $W > "$OUT/${TAG}_bench_$W.log" 2>&1
    rc=$?; echo "[bench $W] rc=$rc"; grep '^{' "$OUT/${TAG}_bench_$W.log" | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
for W in ${WORKLOADS:-uniform zipf queue approx}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$W" -o run -- \
        python3 "$ROOT/bench.py" --workload $W --steps 10 --warmup 3 --cpu-seconds 0 --no-stage-timing --no-pipeline \
        --no-host-buffer --no-strdir > "$OUT/${TAG}_rocprof_$W.log" 2>&1
    rc=$?; echo "[rocprof $W] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
[ "${SKIP_PMC:-0}" = 1 ] && { echo all-done; exit 0; }
bash "$ROOT/tools/pmc_all.sh"
