#!/bin/bash
# round 5: the new GPU tests (config C owners at 8-GPU batch sizes, sync stream ordering, owner-map clamp)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_approx.py::test_sync_stream_orders_after_producer \
  tests/test_gpu_cluster.py::test_route_plan_bad_owner_map_is_bounds_safe > gpurun_out/r05a_small.log 2>&1
rc=$?; echo "small rc=$rc"; tail -3 gpurun_out/r05a_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 780 --timeout-method thread \
  tests/test_gpu_emul_owner.py > gpurun_out/r05a_emul_owner.log 2>&1
rc=$?; echo "emul rc=$rc"; tail -5 gpurun_out/r05a_emul_owner.log; exit $rc
