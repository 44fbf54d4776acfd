#!/bin/bash
# round 5: parity of the reworked digit histogram, then A/B (wave histogram, narrow pass-0
# records) and a kernel trace of the uniform bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sparse.py tests/test_gpu_fold_shapes.py tests/test_gpu_parity.py > gpurun_out/r05e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05e_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=r05 timeout -k 10 500 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05e_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05e_ablate.log | cut -c1-200 | tail -14; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05e_prof_uniform -o run -- \
  python -u bench.py --workload uniform --steps 20 --warmup 5 --no-host-buffer --no-strdir --no-sparse --cpu-seconds 0 \
  > gpurun_out/r05e_prof_uniform.json 2> gpurun_out/r05e_prof_uniform.err
rc=$?; echo "prof rc=$rc"; exit $rc
