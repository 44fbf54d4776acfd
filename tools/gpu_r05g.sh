#!/bin/bash
# round 5: CU split between the partition and fold streams (env TBE_CU_SPLIT), A/B on the
# uniform and zipf benches, two rounds each
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r05g_cusplit.log
for r in 1 2; do
  for w in uniform zipf; do
    for d in 0 8 4 2; do
      TBE_CU_SPLIT=$d timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-host-buffer \
        --no-strdir --no-sparse --cpu-seconds 0 > gpurun_out/r05g_b.json 2> gpurun_out/r05g_b.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w d=$d rc=$rc"; tail -5 gpurun_out/r05g_b.err; exit $rc; }
      python - "$w" "$d" >> gpurun_out/r05g_cusplit.log <<'PY'
import json, sys
l = [json.loads(x) for x in open("gpurun_out/r05g_b.json") if x.startswith("{")][-1]
print(sys.argv[1], "split", sys.argv[2], l["ms_per_step"], json.dumps(l["stage_ms_per_step_overlapped"]))
PY
      tail -1 gpurun_out/r05g_cusplit.log
    done
  done
done
