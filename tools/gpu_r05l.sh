#!/bin/bash
# round 5: sparse fold's chunk fence at workgroup scope (parity), then the sparse-batch gate
# A/B (sweep at 2^21 .. 2^23)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sparse.py \
  > gpurun_out/r05l_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05l_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=gate timeout -k 10 600 python -u tools/ablate.py --run --rounds 2 --steps 5 > gpurun_out/r05l_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep "sweep" gpurun_out/r05l_ablate.log | cut -c1-250; exit $rc
