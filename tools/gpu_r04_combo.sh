#!/bin/bash
# the final tree's config C emulations, then the tools/wip_*.patch experiments: parity
# (TBE_LIB = the patched build) and timing (ABLATE_SET=wipE)
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 400 python -u bench.py --workload zipf --emulate-world 8 --steps 20 --warmup 5 > gpurun_out/r04t_emul8.log 2>&1 || { echo emul8 failed; tail -5 gpurun_out/r04t_emul8.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload zipf --emulate-world 4 --steps 20 --warmup 5 > gpurun_out/r04t_emul4.log 2>&1 || { echo emul4 failed; exit 1; }
TBE_LIB=tools/ablate_libs/libtbe_wip_fused_refresh.so timeout -k 10 400 python -u -m pytest tests/test_gpu_cancel.py tests/test_gpu_approx.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t_fused_tests.log 2>&1; rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/r04t_fused_tests.log; [ $rc -le 1 ] || exit $rc
TBE_LIB=tools/ablate_libs/libtbe_wip_no_memsets.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t_nomemset_tests.log 2>&1; rc=$?; echo "nomemset tests rc=$rc"; tail -2 gpurun_out/r04t_nomemset_tests.log; [ $rc -le 1 ] || exit $rc
TBE_LIB=tools/ablate_libs/libtbe_wip_hot_summary_pipelined.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -k "zipf or hot" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04t_hotpipe_tests.log 2>&1; rc=$?; echo "hotpipe tests rc=$rc"; tail -2 gpurun_out/r04t_hotpipe_tests.log; [ $rc -le 1 ] || exit $rc
ABLATE_SET=wipE ROUNDS=2 STEPS=10 ABLATE_TIMEOUT=500 TAG=r04t bash tools/gpu_r04a.sh ablate
