#!/bin/bash
# round 5: pipelined against serial engines once the timed engine records no stage events
set -o pipefail
mkdir -p gpurun_out
ABLATE_SET=pipe timeout -k 10 600 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05r_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05r_ablate.log | cut -c1-40; exit $rc
