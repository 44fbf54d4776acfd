#!/bin/bash
# round 5: XCD-aware hot-run segments, sparse-batch bounds/dense list by look-back and no
# hot machinery in sparse batches (parity), then the hot A/B and the batch-size sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_emul_owner.py "tests/test_gpu_fullshape.py::test_config_c_slice_full_shape" \
  "tests/test_gpu_fullshape.py::test_key_turns_hot_mid_run" "tests/test_gpu_fullshape.py::test_config_b_full_shape_pipelined" \
  tests/test_gpu_pipeline.py > gpurun_out/r05k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05k_pytest.log; [ $rc -eq 0 ] || exit $rc
ABLATE_SET=hotxcd timeout -k 10 400 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05k_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05k_ablate.log | cut -c1-220 | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload uniform --steps 5 --warmup 2 --no-host-buffer --no-strdir > gpurun_out/r05k_bench_uniform.json 2> gpurun_out/r05k_bench_uniform.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/r05k_bench_uniform.json').read().strip().splitlines()[-1])
for b in d['batch_sweep']: print(b['batch'], b['ms_per_batch'], b['latency_ms'], b['stage_ms_per_batch'])
"; exit $rc
