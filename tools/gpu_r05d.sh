#!/bin/bash
# round 5: config C cold start with the per-batch sampler, then the uniform and zipf bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" > gpurun_out/r05d_fullshape_c.log 2>&1
rc=$?; echo "c rc=$rc"; tail -3 gpurun_out/r05d_fullshape_c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload uniform --steps 20 --warmup 5 --no-host-buffer --no-strdir \
  --cpu-seconds 0 > gpurun_out/r05d_bench_uniform.json 2> gpurun_out/r05d_bench_uniform.err
rc=$?; echo "bench u rc=$rc"; tail -c 300 gpurun_out/r05d_bench_uniform.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload zipf --steps 20 --warmup 5 --no-host-buffer --no-strdir \
  --cpu-seconds 0 > gpurun_out/r05d_bench_zipf.json 2> gpurun_out/r05d_bench_zipf.err
rc=$?; echo "bench z rc=$rc"; tail -c 300 gpurun_out/r05d_bench_zipf.err; exit $rc
