for i in 1 2; do for f in "" "--engine-first"; do
  timeout -k 10 300 python -u bench.py --workload queue --steps 20 --warmup 5 --cpu-seconds 0 --no-host-buffer --no-strdir --no-drain-variant $f > gpurun_out/r06i_q${f}_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06i_q${f}_$i.log') if l.startswith('{')][0]); r=d['roofline']; print('order${f:- default}', $i, d['ms_per_step'], 'timed fold', r['avg_launch_ms'], 'replay fold', d['stage_ms_per_step']['fold'])"
done; done
