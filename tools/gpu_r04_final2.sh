#!/bin/bash
# round 4, last engine change (one-pass one-client refresh): the GPU suite, the hot-summary
# pipelining experiment (parity on its patched build, then timing), and the final bench
# lines with rocprof statistics (tools/gpu_final_r04.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TESTS='tests -m gpu' TAG=r04s bash tools/gpu_r04a.sh tests || exit $?
TBE_LIB=tools/ablate_libs/libtbe_wip_hot_summary_pipelined.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -k "zipf or hot" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04s_hotpipe_tests.log 2>&1; rc=$?; echo "hotpipe tests rc=$rc"; tail -2 gpurun_out/r04s_hotpipe_tests.log; [ $rc -le 1 ] || exit $rc
ABLATE_SET=wipF ROUNDS=2 STEPS=10 ABLATE_TIMEOUT=300 TAG=r04s bash tools/gpu_r04a.sh ablate || exit $?
TAG=r04s SKIP_TESTS=1 bash tools/gpu_final_r04.sh
