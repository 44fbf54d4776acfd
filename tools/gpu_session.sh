set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_dev.log 2>&1; rc=$?; tail -5 gpurun_out/t_dev.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload queue --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/b_queue.log 2>&1; rc=$?; tail -3 gpurun_out/b_queue.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload approx --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/b_approx.log 2>&1; rc=$?; tail -3 gpurun_out/b_approx.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 3 > gpurun_out/b_uni.log 2>&1; rc=$?; tail -3 gpurun_out/b_uni.log
