#!/bin/bash
# round 5: sparse gate at R/8 per bucket (parity up to 2^23), then the A/B of hot runs in
# sparse batches (uniform and Zipf sweeps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py \
  tests/test_gpu_parity.py "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" > gpurun_out/r05m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05m_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=hotmin timeout -k 10 700 python -u tools/ablate.py --run --rounds 2 --steps 5 > gpurun_out/r05m_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep "sweep" gpurun_out/r05m_ablate.log | cut -c1-130; exit $rc
