set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/final_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/final_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?; tail -1 gpurun_out/final_smoke.log
timeout -k 10 420 python -u bench.py > gpurun_out/final_bench.log 2>&1 || exit $?; grep '^{' gpurun_out/final_bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_final -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-stage-timing --no-pipeline --no-host-buffer > $GRAFT_REPO_ROOT/gpurun_out/final_rocprof.log 2>&1 || exit $?
echo final-done
