#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/diag_b2b_queue2.py > gpurun_out/r05z6_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/r05z6_diag.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
TBE_LIB=$PWD/tools/ablate_libs/libtbe_TBE_Q_REG_SLICE1.so timeout -k 10 400 python -u tools/diag_b2b_queue2.py > gpurun_out/r05z6_diag_qreg.log 2>&1
rc=$?; echo "diag qreg rc=$rc"; grep -v amdgpu.ids gpurun_out/r05z6_diag_qreg.log | cut -c1-250; exit $rc
