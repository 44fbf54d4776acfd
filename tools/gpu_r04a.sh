#!/bin/bash
# round 4, first GPU session: the changed/new GPU tests, then the config C owner emulation
# and a config B bench line with the sparse-batch leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
timeout -k 10 1500 python -u -m pytest tests/test_gpu_dist_large.py tests/test_gpu_cluster.py tests/test_gpu_dist.py \
    tests/test_gpu_approx.py tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_gpu_fold_shapes.py \
    -q -rf --timeout 400 --timeout-method thread > $OUT/r04a_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 $OUT/r04a_pytest.log
# 1 = failed tests (read the log); anything else (timeout, crash, fault) ends the session
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --workload zipf --emulate-world 8 --steps 20 --warmup 5 > $OUT/r04a_emul8.log 2>&1 || { echo "emul8 failed"; tail -20 $OUT/r04a_emul8.log; exit 1; }
tail -c 3000 $OUT/r04a_emul8.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/r04a_bench_uniform.log 2>&1 || { echo "bench failed"; tail -20 $OUT/r04a_bench_uniform.log; exit 1; }
tail -c 1500 $OUT/r04a_bench_uniform.log
