#!/bin/bash
# Diagnostic (round 6): one rocprofv3 --pmc pass of SQ instruction counters over a short
# bench run (3 timed batches), per-kernel CSV under gpurun_out/<name>/.
#   bash tools/diag/sq_pass.sh <name> <bench.py args...>
# then: python tools/diag/sq_summary.py gpurun_out/<name>/run_counter_collection.csv <kernel substring>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
name=$1
shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM \
    SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d "$ROOT/gpurun_out/$name" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-host-buffer --no-strdir "$@"
