#!/bin/bash
# round 5: the sampler without 64-bit divisions (parity of the hot paths), then the A/B of
# hot runs in sparse batches >= 2^20 (uniform and Zipf sweeps, plus the dense 2^26 lines)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_key_turns_hot_mid_run" "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" \
  tests/test_gpu_emul_owner.py tests/test_gpu_sparse.py tests/test_gpu_parity.py > gpurun_out/r05q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05q_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=hotmin timeout -k 10 700 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05q_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05q_ablate.log | cut -c1-110; exit $rc
