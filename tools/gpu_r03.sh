#!/bin/bash
# Round-3 GPU session: the GPU suite (new world-2 tests first), smoke, a two-rank
# rehearsal of bench.py --gpus 2 on the one GPU (--share-device), and the bench lines.
# Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r03a}
step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; tail -3 "$OUT/${TAG}_${name}.log"
    [ $rc -ne 0 ] && exit $rc
    return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || {
[ "${DIST:-0}" = 1 ] && step pytest_dist 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
}
[ "${SKIP_REHEARSAL:-0}" = 1 ] || {
step rehearse_uniform 300 python -u bench.py --gpus 2 --share-device --keys 10000000 --batch 4194304 --steps 3 --warmup 1 --cpu-seconds 0
step rehearse_approx 300 python -u bench.py --gpus 2 --share-device --workload approx --keys 1000000 --batch 4194304 --steps 3 --warmup 1 --cpu-seconds 0
step rehearse_queue 300 python -u bench.py --gpus 2 --share-device --workload queue --keys 10000000 --batch 4194304 --steps 3 --warmup 1 --cpu-seconds 0
}
for W in ${BENCH:-uniform}; do
    step bench_$W 400 python -u bench.py --workload $W --steps 20 --warmup 5
done
[ -n "${PMC:-}" ] && { WORKLOADS="$PMC" timeout -k 10 900 bash tools/pmc_passes.sh > "$OUT/${TAG}_pmc.log" 2>&1; rc=$?; echo "[pmc] rc=$rc"; tail -3 "$OUT/${TAG}_pmc.log"; [ $rc -ne 0 ] && exit $rc; }
echo all-done
