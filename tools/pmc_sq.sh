#!/bin/bash
# One SQ-counter pass (wave cycles split into parked / issue-stalled / active, LDS and
# VALU instruction counts, LDS bank conflicts) over a short bench run of one workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
W=${WORKLOAD:-uniform}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$OUT/pmcsq_$W" -o run -- \
    python3 "$ROOT/bench.py" --workload $W --steps 2 --warmup 1 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer --no-strdir \
    > "$OUT/pmcsq_$W.log" 2>&1
rc=$?; echo "[pmc sq $W] rc=$rc"; exit $rc
