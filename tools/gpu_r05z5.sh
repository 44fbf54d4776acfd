#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/diag_poison.py > gpurun_out/r05z5_poison.log 2>&1
rc=$?; echo "poison rc=$rc"; grep -v amdgpu.ids gpurun_out/r05z5_poison.log | cut -c1-250; exit $rc
