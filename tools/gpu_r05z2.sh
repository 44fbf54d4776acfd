#!/bin/bash
# round 5 (second session): pipelined queue kind + many-workgroup hot sampler.  Targeted
# parity tests on the new build first, then the same-box A/B (three rounds).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_device_queue.py tests/test_gpu_pipeline.py tests/test_gpu_queue.py \
  "tests/test_gpu_fullshape.py::test_key_turns_hot_mid_run" "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" "tests/test_gpu_fullshape.py::test_config_d_full_shape" \
  tests/test_gpu_sparse.py > gpurun_out/r05z2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05z2_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=r05b timeout -k 10 1000 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05z2_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05z2_ablate.log | cut -c1-60; exit $rc
