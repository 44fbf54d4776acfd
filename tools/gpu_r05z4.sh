#!/bin/bash
# round 5: back-to-back queue diagnostic on the working tree's engine and on HEAD's
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/diag_b2b_queue.py > gpurun_out/r05z4_diag_new.log 2>&1
rc=$?; echo "diag new rc=$rc"; grep -v amdgpu.ids gpurun_out/r05z4_diag_new.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
TBE_LIB=$PWD/tools/ablate_libs/libtbe_head.so timeout -k 10 400 python -u tools/diag_b2b_queue.py > gpurun_out/r05z4_diag_head.log 2>&1
rc=$?; echo "diag head rc=$rc"; grep -v amdgpu.ids gpurun_out/r05z4_diag_head.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=r05q timeout -k 10 700 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05z4_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05z4_ablate.log | cut -c1-60; exit $rc
