#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run, as MI355X_MICROARCH.md prescribes)
# over (a) the counter calibration patterns (tools/pmc_calib.py) and (b) the benchmark
# exactly as the driver runs it (bench.py --steps 20 --warmup 5; the summary keeps only
# the dispatches between the k_mark<1> / k_mark<2> markers around the timed batches).
# CSVs land in gpurun_out/pmc3_<run>_<pass>/ for tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_32B TCC_EA0_RDREQ"
  "TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ_64B TCC_EA0_WRREQ"
)
run() {   # run <name> <secs> <cmd...>
    local name=$1 secs=$2; shift 2
    for i in "${!PASSES[@]}"; do
        # the bench run records its configuration (bench_kinds.run_fingerprint) for the summary
        TBE_PMC_FINGERPRINT="$OUT/pmc3_${name}_fingerprint.json" timeout -s KILL "$secs" rocprofv3 --pmc ${PASSES[$i]} --output-format csv -d "$OUT/pmc3_${name}_p$i" -o run -- \
            "$@" > "$OUT/pmc3_${name}_p$i.log" 2>&1
        local rc=$?
        echo "[pmc $name pass $i] rc=$rc"
        if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc3_${name}_p$i.log"; exit $rc; fi
    done
}
[ "${SKIP_CALIB:-0}" = 1 ] || run calib 120 python3 "$ROOT/tools/pmc_calib.py"
for W in ${WORKLOADS:-uniform}; do
    if [ "$W" = queue_draining ]; then   # config D's draining schedule (the markers go around it)
        run $W 300 python3 "$ROOT/bench.py" --workload queue --steps 20 --warmup 5 --cpu-seconds 0 \
            --no-stage-timing --no-host-buffer --no-strdir --drain-marked
        continue
    fi
    run $W 240 python3 "$ROOT/bench.py" --workload $W --steps 20 --warmup 5 --cpu-seconds 0 \
        --no-stage-timing --no-host-buffer --no-strdir --no-sparse --no-drain-variant
done
echo pmc-done
