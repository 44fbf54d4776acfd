#!/bin/bash
# round 5: the replenish tick skips no-op writing passes (parity of the queue paths), then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_queue.py \
  tests/test_gpu_device_queue.py tests/test_gpu_cancel.py "tests/test_gpu_fullshape.py::test_config_d_full_shape" \
  > gpurun_out/r05x_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05x_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=tick timeout -k 10 700 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05x_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05x_ablate.log | cut -c1-200; exit $rc
