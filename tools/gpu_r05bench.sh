#!/bin/bash
# round 5 final: smoke, the four bench lines (PMC bytes attached when the committed
# profiles/pmc_summary.json matches) and rocprofv3 kernel statistics of config B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=r05zz SKIP_TESTS=1 PROF="uniform" DRIVER_PROF=0 timeout -k 10 1100 bash tools/gpu_final_r05.sh
