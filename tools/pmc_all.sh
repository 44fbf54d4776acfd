#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE: one counter group per run, as
# MI355X_MICROARCH.md prescribes) over short bench runs of every workload; CSVs land in
# gpurun_out/pmc_<workload>_<counter>/ for tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for W in ${WORKLOADS:-uniform zipf queue approx}; do
    for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${W}_$C" -o run -- \
            python3 "$ROOT/bench.py" --workload $W --steps 2 --warmup 1 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer --no-strdir \
            > "$OUT/pmc_${W}_$C.log" 2>&1
        rc=$?
        echo "[pmc $W $C] rc=$rc"
        if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_${W}_$C.log"; exit $rc; fi
    done
done
echo pmc-done
