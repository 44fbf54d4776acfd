#!/bin/bash
# Diagnostic (round 6): config B's fold, the pre-12-byte-row engine (tools/ablate_libs/
# libtbe_r06pre.so) against the tree's, on one box: bench lines alternated, then one
# rocprofv3 --pmc pass of SQ instruction counters per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r06g}
ARGS="--workload uniform --steps 10 --warmup 3 --cpu-seconds 0 --no-host-buffer --no-strdir --no-sparse"
for i in 1 2; do
  for v in r06pre tree; do
    lib=$ROOT/distributedratelimiting.redis_amd/libtbe.so
    [ $v = r06pre ] && lib=$ROOT/tools/ablate_libs/libtbe_r06pre.so
    TBE_LIB=$lib timeout -k 10 200 python -u bench.py $ARGS > $OUT/${TAG}_ab_${v}_$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/${TAG}_ab_${v}_$i.log') if l.startswith('{')][0]); print('$v', $i, d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in r06pre tree; do
  lib=$ROOT/distributedratelimiting.redis_amd/libtbe.so
  [ $v = r06pre ] && lib=$ROOT/tools/ablate_libs/libtbe_r06pre.so
  TBE_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
     --output-format csv -d $OUT/${TAG}_pmc_$v -o run -- python3 $ROOT/bench.py --workload uniform --steps 3 --warmup 1 --cpu-seconds 0 --no-host-buffer --no-strdir --no-sparse > $OUT/${TAG}_pmc_$v.log 2>&1 || exit $?
  echo "pmc $v done"
done
