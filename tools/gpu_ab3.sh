#!/bin/bash
# A/B bench lines: the same workload with and without a flag, alternating, each under its
# own time limit.  AB_FLAG is the bench flag of the B side; WORKLOADS the workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-ab3}
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
    rc=$?; tail -3 "$OUT/${TAG}_tests.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for W in ${WORKLOADS:-uniform}; do
    for side in A B; do
      flag=""; [ $side = B ] && flag="$AB_FLAG"
      timeout -k 10 300 python -u bench.py --workload $W --steps ${STEPS:-20} --warmup 5 --cpu-seconds 0 --no-host-buffer --no-strdir --no-drain-variant $flag > "$OUT/${TAG}_${W}_${side}_$r.log" 2>&1
      rc=$?
      [ $rc -ne 0 ] && { echo "[$W $side] rc=$rc"; tail -5 "$OUT/${TAG}_${W}_${side}_$r.log"; exit $rc; }
      python3 - "$OUT/${TAG}_${W}_${side}_$r.log" $W $side <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][0]
d = json.loads(l)
print(sys.argv[2], sys.argv[3], d["ms_per_step"], json.dumps(d["stage_ms_per_step"]))
PY
    done
  done
done
echo ab-done
