#!/bin/bash
# Round-2 GPU session: full GPU suite, full-shape parity gate, the streaming-hint
# experiment on the dense approximate fold, default bench, rocprof stats, PMC passes.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
stop() { echo "[stop] $1 rc=$2"; exit "$2"; }
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }

if [ "${WALK_FIRST:-0}" = 1 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 200 --timeout-method thread \
    > "$OUT/r02_walk.log" 2>&1
rc=$?; tail -3 "$OUT/r02_walk.log"; [ $rc -ne 0 ] && stop walk $rc
fi
if [ "${SKIP_SUITE:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    --ignore=tests/test_gpu_fullshape.py > "$OUT/r02_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/r02_pytest_gpu.log"; fatal $rc && stop suite $rc
fi
if [ "${SKIP_FULL:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullshape.py -x -v -s --timeout 900 --timeout-method thread \
    > "$OUT/r02_fullshape.log" 2>&1
rc=$?; grep -E "fullshape|passed|failed|Error" "$OUT/r02_fullshape.log" | tail -30; fatal $rc && stop fullshape $rc
fi
if [ "${NT_EXP:-1}" = 1 ]; then
for v in nt plain; do
    TBE_LIB=$ROOT/tools/ablate_libs/libtbe_TBE_APPROX_DENSE$( [ $v = plain ] && echo _TBE_APPROX_DENSE_PLAIN).so timeout -k 10 300 python -u -m pytest \
        tests/test_gpu_approx.py -q -k "clients_epochs" --timeout 120 --timeout-method thread \
        > "$OUT/r02_nt_exp_$v.log" 2>&1
    rc=$?; echo "[nt-exp $v] rc=$rc"; tail -3 "$OUT/r02_nt_exp_$v.log"; fatal $rc && stop nt-exp $rc
done
fi
if [ "${ABLATE:-0}" = 1 ]; then
timeout -k 10 900 python -u tools/ablate.py --run --rounds 1 --steps 5 > "$OUT/r02_ablate.log" 2>&1
rc=$?; echo "[ablate] rc=$rc"; grep -E "^[0-9] " "$OUT/r02_ablate.log" | cut -c1-400; fatal $rc && stop ablate $rc
fi
[ "${SKIP_BENCH:-0}" = 1 ] && { echo r02-done; exit 0; }
timeout -k 10 420 python -u bench.py > "$OUT/r02_bench.log" 2>&1
rc=$?; grep '^{' "$OUT/r02_bench.log" | cut -c1-400; fatal $rc && stop bench $rc
[ $rc -ne 0 ] && stop bench $rc
[ "${SKIP_PROF:-0}" = 1 ] && { echo r02-done; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r02_prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer --no-strdir \
    > "$OUT/r02_rocprof.log" 2>&1
rc=$?; echo "[rocprof] rc=$rc"; [ $rc -ne 0 ] && stop rocprof $rc
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_uniform_$C" -o run -- \
        python3 "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer --no-strdir \
        > "$OUT/pmc_uniform_$C.log" 2>&1
    rc=$?; echo "[pmc $C] rc=$rc"; [ $rc -ne 0 ] && stop pmc $rc
done
echo r02-done
