set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for K in 50000000 25000000 12500000; do
  timeout -k 10 300 python -u bench.py --keys $K --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/scale_$K.log 2>&1 || exit $?
  python -c "
import json;d=json.loads([l for l in open('gpurun_out/scale_$K.log') if l.startswith('{')][0])
print($K, '%.3e'%d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['config']['layout'])"
done
