#!/bin/bash
# round 5: the timed engine without stage events (A/B)
set -o pipefail
mkdir -p gpurun_out
ABLATE_SET=events timeout -k 10 600 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05o_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05o_ablate.log | cut -c1-60; exit $rc
