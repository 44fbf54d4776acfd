#!/bin/bash
# Round-5 session: the whole GPU suite (as the driver runs it), smoke(), the four
# bench lines, and a rocprofv3 --kernel-trace --stats run of each bench (kernel statistics
# for profiles/); with PMC=1 also the counter passes of tools/pmc_passes.sh.  Each step under
# its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05z}
step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; tail -2 "$OUT/${TAG}_${name}.log"
    [ $rc -ne 0 ] && exit $rc
    return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || {
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
}
for W in ${BENCH:-uniform zipf queue approx}; do
    step bench_$W 400 python -u bench.py --workload $W --steps 20 --warmup 5
done
[ "${SKIP_PROF:-0}" = 1 ] || {
cd /tmp && export TMPDIR=/tmp
for W in ${PROF:-uniform zipf queue approx}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_$W" -o run -- \
        python3 "$ROOT/bench.py" --workload $W --steps 20 --warmup 5 --cpu-seconds 0 --no-host-buffer \
        --no-strdir > "$OUT/${TAG}_prof_$W.log" 2>&1
    rc=$?; echo "[prof $W] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/${TAG}_prof_$W.log"; exit $rc; }
done
# the driver's exact command line (its kernel statistics include the host-buffer and
# string-directory legs that run after the timed region)
[ "${DRIVER_PROF:-1}" = 1 ] && {
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof_driver" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 > "$OUT/${TAG}_prof_driver.log" 2>&1
rc=$?; echo "[prof driver] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/${TAG}_prof_driver.log"; exit $rc; }
}
cd "$ROOT"
}
if [ "${PMC:-0}" = 1 ]; then
    SKIP_CALIB=${SKIP_CALIB:-1} WORKLOADS="${PMC_WORKLOADS:-uniform zipf queue approx}" \
        timeout -k 10 1000 bash tools/pmc_passes.sh > "$OUT/${TAG}_pmc.log" 2>&1
    rc=$?; echo "[pmc] rc=$rc"; tail -2 "$OUT/${TAG}_pmc.log"; [ $rc -ne 0 ] && exit $rc
fi
echo all-done
