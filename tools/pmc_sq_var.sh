#!/bin/bash
# SQ-counter pass (tools/pmc_sq.sh counters) over each ablation build in tools/ablate_libs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$ROOT"/tools/ablate_libs/*.so; do
    V=$(basename "$L" .so)
    TBE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        --output-format csv -d "$OUT/pmcsq_$V" -o run -- \
        python3 "$ROOT/bench.py" --workload ${WORKLOAD:-uniform} --steps 2 --warmup 1 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer --no-strdir \
        > "$OUT/pmcsq_$V.log" 2>&1
    rc=$?; echo "[pmc sq $V] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
