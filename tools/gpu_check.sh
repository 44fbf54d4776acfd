#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench, and a rocprofv3 kernel trace.
# Stops at the first step that faults, aborts or times out (rc not in {0,1}).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-5}
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
export PYTHONUNBUFFERED=1
step pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python -u bench.py --steps "$STEPS" --warmup 2 --cpu-seconds 8
if [ "${PROFILE:-1}" = "1" ]; then
    cd /tmp && export TMPDIR=/tmp
    step rocprof 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer
    cd "$ROOT"
fi
echo done
