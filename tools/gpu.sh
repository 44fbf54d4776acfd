#!/bin/bash
# The one GPU-box launcher (round 6; it replaces rounds 2-5's one-off tools/gpu_*.sh).
#
#   TAG=r06a bash tools/gpu.sh <step> [<step> ...]
#
# Each step runs under its own time limit; its output goes to gpurun_out/<TAG>_<name>.log.
# A step that fails, faults, aborts or times out ends the script with its exit status, so
# nothing else touches the GPU after it.  Steps:
#
#   suite                 pytest -m gpu (the driver's command) + smoke()
#   test:<path>[::<id>]   one GPU test file / test (e.g. test:tests/test_gpu_recreate.py)
#   smoke                 __graft_entry__.smoke()
#   bench:<workload>      bench.py --workload <workload> --steps 20 --warmup 5 (BENCH_ARGS appended)
#   driver                bench.py --steps 20 --warmup 5, as the driver runs it
#   prof:<workload>       rocprofv3 --kernel-trace --stats of that bench (CSV under gpurun_out/<TAG>_prof_<w>/)
#   pmc:<w1,w2,...>       rocprofv3 --pmc passes (tools/pmc_passes.sh) + tools/pmc_summary.py
#   ablate:<set>          ABLATE_SET=<set> tools/ablate.py --run (variants built here first; ABLATE_ARGS appended)
#   alias:<trials>:<mask> tools/diag/contig_alias (contiguous-allocation aliasing check)
#   cmd:<name>:<secs>:<command>   anything else
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06}
PYTEST="python -u -m pytest -x -v --timeout 600 --timeout-method thread"

step() {   # step <name> <seconds> <command string>
    local name=$1 secs=$2 cmd=$3 t0
    t0=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 3 "$OUT/${TAG}_${name}.log" | cut -c1-400
    [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}

prof() {   # rocprofv3 with the program itself after -- (no launcher hop)
    local w=$1
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/${TAG}_prof_$w" -o run -- python3 "$ROOT/bench.py" --workload "$w" --steps 20 --warmup 5 \
        --cpu-seconds 0 --no-host-buffer --no-strdir ) > "$OUT/${TAG}_prof_$w.log" 2>&1
    local rc=$?
    echo "[prof:$w] rc=$rc"
    tail -n 2 "$OUT/${TAG}_prof_$w.log" | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
    # kernel statistics and the timed / replay marker windows, for profiles/
    cp "$OUT/${TAG}_prof_$w/run_kernel_stats.csv" "$OUT/${TAG}_${w}_kernel_stats.csv" 2>/dev/null
    python3 tools/prof_window.py "$OUT/${TAG}_prof_$w/run_kernel_trace.csv" \
        --out "$OUT/${TAG}_${w}_kernel_windows.json" > "$OUT/${TAG}_${w}_kernel_windows.txt" 2>&1 || true
}

for s in "$@"; do
    case "$s" in
        suite)
            step pytest_gpu 1500 "$PYTEST tests -m gpu"
            step smoke 300 "python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
        smoke)
            step smoke 300 "python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
        test:*)
            t=${s#test:}; n=$(basename "${t%%::*}" .py)
            step "$n" 900 "$PYTEST '$t'" ;;
        bench:*)
            w=${s#bench:}
            step "bench_$w" 500 "python -u bench.py --workload $w --steps 20 --warmup 5 ${BENCH_ARGS:-}" ;;
        driver)
            step bench_driver 500 "python -u bench.py --steps 20 --warmup 5" ;;
        prof:*)
            prof "${s#prof:}" ;;
        pmc:*)
            w=${s#pmc:}
            step pmc 1400 "SKIP_CALIB=${SKIP_CALIB:-1} WORKLOADS='${w//,/ }' bash tools/pmc_passes.sh"
            step pmc_summary 120 "python3 tools/pmc_summary.py --write && cp profiles/pmc_summary.json $OUT/${TAG}_pmc_summary.json" ;;
        ablate:*)
            step "ablate_${s#ablate:}" 1400 "ABLATE_SET=${s#ablate:} python -u tools/ablate.py --run ${ABLATE_ARGS:-}" ;;
        alias:*)
            a=${s#alias:}
            step "alias_${a//:/_}" 600 "tools/diag/contig_alias ${a%%:*} ${a#*:}" ;;
        cmd:*)
            r=${s#cmd:}; n=${r%%:*}; r=${r#*:}; secs=${r%%:*}; c=${r#*:}
            step "$n" "$secs" "$c" ;;
        *)
            echo "unknown step $s"; exit 2 ;;
    esac
done
echo all-done
