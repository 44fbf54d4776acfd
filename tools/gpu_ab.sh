#!/bin/bash
# Ablation session: parity of the default build on the fold tests, then tools/ablate.py
# (variants built beforehand with `python tools/ablate.py --build`).  Each GPU step has
# its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-ab}
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
    rc=$?; tail -3 "$OUT/${TAG}_tests.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 env ABLATE_SET=${ABLATE_SET:-queue} python -u tools/ablate.py --run --rounds ${ROUNDS:-1} --steps ${STEPS:-10} > "$OUT/${TAG}_ablate.log" 2>&1
rc=$?; grep -E "^[0-9] |FAILED" "$OUT/${TAG}_ablate.log" | cut -c1-600; exit $rc
