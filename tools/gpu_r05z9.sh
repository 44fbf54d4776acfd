#!/bin/bash
# round 5: the back-to-back queue diagnostic with contiguous rings and with ordinary rings,
# alternating, on one box
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for v in TBE_CONTIG_ALLOC4 base; do
    TBE_LIB=$PWD/tools/ablate_libs/libtbe_$v.so timeout -k 10 300 python -u tools/diag_b2b_queue.py > gpurun_out/r05z9_diag_${v}_$i.log 2>&1
    rc=$?; echo "== $v round $i rc=$rc"; grep "^lib=" gpurun_out/r05z9_diag_${v}_$i.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
  done
done
