#!/bin/bash
# round 5: the whole GPU suite on the current tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05f_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r05f_pytest_gpu.log; exit $rc
