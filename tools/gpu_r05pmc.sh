#!/bin/bash
# round 5 final: PMC passes (calibration + the four benches as the driver runs them) and
# their summary on the box (profiles/pmc_summary.json, copied to gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SKIP_CALIB=0 WORKLOADS="uniform zipf queue approx" timeout -k 10 1100 bash tools/pmc_passes.sh > gpurun_out/r05zz_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/r05zz_pmc.log; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py --write > gpurun_out/r05zz_pmc_summary.txt 2>&1
rc=$?; echo "summary rc=$rc"; tail -5 gpurun_out/r05zz_pmc_summary.txt; cp profiles/pmc_summary.json gpurun_out/r05zz_pmc_summary.json; exit $rc
