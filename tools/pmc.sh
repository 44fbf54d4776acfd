#!/bin/bash
# PMC passes (one counter group per run, as MI355X_MICROARCH.md prescribes) over a short
# bench run; CSVs land in gpurun_out/pmc_<pass>/.  Usage: [BENCH_ARGS=...] bash tools/pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {  # pass NAME COUNTERS...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --no-stage-timing ${BENCH_ARGS:-} \
        > "$OUT/pmc_$name.log" 2>&1
    local rc=$?
    echo "[pmc $name] rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$name.log"; exit $rc; fi
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
pass valu SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT
echo pmc-done
