#!/bin/bash
# round 5 (second session): diagnose the serial back-to-back queue mismatch, then the
# same-box A/B of the sampler and the queue pipeline (three rounds).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/diag_b2b_queue.py > gpurun_out/r05z3_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/r05z3_diag.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=r05b timeout -k 10 1000 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05z3_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05z3_ablate.log | cut -c1-60; exit $rc
