#!/bin/bash
# round 5: the fold at two workgroups per CU (LDS pad) with/without pass 0's hot table
# aliased into its staging buffer, so partition workgroups fit beside the fold
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ABLATE_SET=r05s timeout -k 10 1000 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05z7_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05z7_ablate.log | cut -c1-70; exit $rc
