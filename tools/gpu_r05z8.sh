#!/bin/bash
# round 5: the whole GPU suite on ordinary (non-contiguous) rings, smoke, then the
# fold-at-two-workgroups-per-CU A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/r05z8_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r05z8_pytest_gpu.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z8_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r05z8_smoke.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=r05s timeout -k 10 900 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05z8_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05z8_ablate.log | cut -c1-70; exit $rc
