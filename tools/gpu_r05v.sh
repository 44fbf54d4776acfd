#!/bin/bash
# round 5: the small sampler (parity of the hot paths), then its A/B against the 133 KB one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_key_turns_hot_mid_run" "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" \
  tests/test_gpu_emul_owner.py tests/test_gpu_sparse.py tests/test_gpu_parity.py > gpurun_out/r05v_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05v_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=hs timeout -k 10 700 python -u tools/ablate.py --run --rounds 3 --steps 20 > gpurun_out/r05v_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05v_ablate.log | cut -c1-60; exit $rc
