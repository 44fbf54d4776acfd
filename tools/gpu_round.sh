#!/bin/bash
# tests + smoke + bench (+rocprof) then fold ablation; stops on fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PROFILE=${PROFILE:-1} bash tools/gpu_check.sh || exit $?
timeout -k 10 600 python -u tools/ablate.py --run --rounds ${ABLATE_ROUNDS:-1} --steps 5 > gpurun_out/ablate.log 2>&1
rc=$?; echo "[ablate] rc=$rc"; tail -6 gpurun_out/ablate.log | cut -c1-300
