#!/bin/bash
# round 5: config E 8-client full shape, then the uniform and approx bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 480 --timeout-method thread \
  "tests/test_gpu_fullshape.py::test_config_e_full_shape_eight_clients" > gpurun_out/r05c_fullshape_e8.log 2>&1
rc=$?; echo "e8 rc=$rc"; tail -3 gpurun_out/r05c_fullshape_e8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload uniform --steps 20 --warmup 5 --no-host-buffer --no-strdir \
  --cpu-seconds 0 > gpurun_out/r05c_bench_uniform.json 2> gpurun_out/r05c_bench_uniform.err
rc=$?; echo "bench u rc=$rc"; tail -c 400 gpurun_out/r05c_bench_uniform.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload approx --steps 20 --warmup 5 \
  --cpu-seconds 0 > gpurun_out/r05c_bench_approx.json 2> gpurun_out/r05c_bench_approx.err
rc=$?; echo "bench a rc=$rc"; tail -c 400 gpurun_out/r05c_bench_approx.err; exit $rc
