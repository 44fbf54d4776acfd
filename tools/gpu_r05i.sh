#!/bin/bash
# round 5: pass 0's inverse by runs -- parity of the token-bucket paths, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fold_shapes.py tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_emul_owner.py \
  tests/test_gpu_pipeline.py tests/test_gpu_pinned.py "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" \
  "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" > gpurun_out/r05i_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05i_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=unruns timeout -k 10 500 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05i_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05i_ablate.log | cut -c1-220 | tail -10; exit $rc
