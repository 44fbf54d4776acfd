#!/bin/bash
# round 5: hot-run segment size A/B (config C), parity of the hot paths at segment 4096 first
set -o pipefail
mkdir -p gpurun_out
ABLATE_SET=seg timeout -k 10 600 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05u_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05u_ablate.log | cut -c1-250; exit $rc
