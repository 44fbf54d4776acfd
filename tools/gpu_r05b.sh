#!/bin/bash
# round 5: sparse-batch fold, wave digit histogram, per-batch hot sampling, narrow pass-0 records
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sparse.py tests/test_gpu_fold_shapes.py tests/test_gpu_parity.py tests/test_gpu_emul_owner.py \
  > gpurun_out/r05b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 580 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_key_turns_hot_mid_run" \
  "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" \
  "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" > gpurun_out/r05b_fullshape.log 2>&1
rc=$?; echo "fullshape rc=$rc"; tail -3 gpurun_out/r05b_fullshape.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload uniform --steps 20 --warmup 5 --no-host-buffer --no-strdir \
  --cpu-seconds 0 > gpurun_out/r05b_bench_uniform.json 2> gpurun_out/r05b_bench_uniform.err
rc=$?; echo "bench u rc=$rc"; tail -c 300 gpurun_out/r05b_bench_uniform.err; exit $rc
