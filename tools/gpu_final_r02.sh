#!/bin/bash
# Round-2 final session: the whole GPU suite (as the driver runs it), the full-shape
# parity gate and smoke(); each step under its own time limit, a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r02f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/${TAG}_smoke.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_smoke.log"; exit $rc
