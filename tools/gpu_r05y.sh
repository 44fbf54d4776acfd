#!/bin/bash
# round 5: physically contiguous resident state (A/B), four rounds (config D is bimodal)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_queue.py tests/test_gpu_approx.py \
  "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" > gpurun_out/r05yab2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05yab2_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=contig timeout -k 10 900 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05yab2_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05yab2_ablate.log | cut -c1-40; exit $rc
