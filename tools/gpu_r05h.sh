#!/bin/bash
# round 5: A/B (CU split between the partition and fold streams; persistent last pass),
# then the approx (8-client refresh) and queue bench lines
set -o pipefail
mkdir -p gpurun_out
ABLATE_SET=r05b timeout -k 10 700 python -u tools/ablate.py --run --rounds 2 --steps 20 > gpurun_out/r05h_ablate.log 2>&1
rc=$?; echo "ablate rc=$rc"; grep -v "^{" gpurun_out/r05h_ablate.log | cut -c1-220 | tail -18; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload approx --steps 20 --warmup 5 --cpu-seconds 0 \
  > gpurun_out/r05h_bench_approx.json 2> gpurun_out/r05h_bench_approx.err
rc=$?; echo "approx rc=$rc"; tail -c 300 gpurun_out/r05h_bench_approx.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload queue --steps 20 --warmup 5 --cpu-seconds 0 \
  > gpurun_out/r05h_bench_queue.json 2> gpurun_out/r05h_bench_queue.err
rc=$?; echo "queue rc=$rc"; tail -c 300 gpurun_out/r05h_bench_queue.err; exit $rc
