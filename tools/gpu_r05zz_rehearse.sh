#!/bin/bash
# round 5 final tree: two-rank rehearsal of the benches on one GPU (gloo, --share-device)
set -o pipefail
mkdir -p gpurun_out
for w in uniform zipf queue approx; do
  timeout -k 10 300 python -u bench.py --gpus 2 --share-device --workload $w --steps 3 --warmup 1 --cpu-seconds 0 \
    --no-host-buffer --no-strdir --no-sparse > gpurun_out/r05zz_rehearse_$w.json 2> gpurun_out/r05zz_rehearse_$w.err || { echo "$w failed"; tail -20 gpurun_out/r05zz_rehearse_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05zz_rehearse_$w.json').read().strip().splitlines()[-1])
print('$w', d['n_gpus'], d['value'], d['ms_per_step'], d.get('rehearsal'), (d.get('roofline') or {}).get('avg_launch_ms'))"
done
