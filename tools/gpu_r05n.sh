#!/bin/bash
# round 5: kernel trace of 2^20-request sparse batches with and without hot runs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 20 40; do
  TBE_LIB=tools/ablate_libs/libtbe_TBE_HOT_SPARSE_MIN_LOG2$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/r05n_prof_hm$v -o run -- python3 bench.py --workload uniform --steps 2 --warmup 1 --no-host-buffer \
    --no-strdir --cpu-seconds 0 --sweep-log2 20 > gpurun_out/r05n_hm$v.json 2> gpurun_out/r05n_hm$v.err || exit $?
  echo "hm$v done"
done
