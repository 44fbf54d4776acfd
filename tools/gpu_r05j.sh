#!/bin/bash
# round 5: k_hist_dig's tile bounds in parallel (parity), then tile-size / hist_dig A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_sparse.py "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" \
  "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" > gpurun_out/r05j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05j_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=tiles timeout -k 10 600 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05j_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05j_ablate.log | cut -c1-220 | tail -14; exit $rc
