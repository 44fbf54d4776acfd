#!/bin/bash
# round 4 GPU sessions.  part "tests": the changed/new GPU tests; part "bench": the config C
# owner emulation at 8 and 4 GPUs and a config B bench line with the sparse-batch leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
PART=${1:-tests}
TAG=${TAG:-r04a}
if [ "$PART" = tests ]; then
    timeout -k 10 1080 python -u -m pytest ${TESTS:-tests/test_gpu_dist_large.py tests/test_gpu_cluster.py tests/test_gpu_dist.py \
        tests/test_gpu_approx.py tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_gpu_fold_shapes.py \
        tests/test_gpu_fullshape.py tests/test_gpu_pipeline.py tests/test_gpu_pinned.py} \
        -v -rf --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
    rc=$?
    echo "pytest rc=$rc"
    grep -E "passed|failed|FAILED|ERROR" $OUT/${TAG}_pytest.log | tail -15
    exit $rc
fi
if [ "$PART" = bench ]; then
    timeout -k 10 420 python -u bench.py --workload zipf --emulate-world 8 --steps 20 --warmup 5 > $OUT/${TAG}_emul8.log 2>&1 || { echo "emul8 failed"; tail -20 $OUT/${TAG}_emul8.log; exit 1; }
    tail -c 600 $OUT/${TAG}_emul8.log
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/${TAG}_bench_uniform.log 2>&1 || { echo "bench failed"; tail -20 $OUT/${TAG}_bench_uniform.log; exit 1; }
    tail -c 1500 $OUT/${TAG}_bench_uniform.log
    timeout -k 10 300 python -u bench.py --workload zipf --emulate-world 4 --steps 20 --warmup 5 > $OUT/${TAG}_emul4.log 2>&1 || { echo "emul4 failed"; tail -20 $OUT/${TAG}_emul4.log; exit 1; }
    tail -c 600 $OUT/${TAG}_emul4.log
fi
if [ "$PART" = qab ]; then
    # config D on one box: round 2's final tree (tools/r02tree, git worktree of d10368e, built
    # here) and this tree, on the driver's schedule, twice each, alternating
    for r in 1 2; do
        (cd tools/r02tree && timeout -k 10 240 python -u bench.py --workload queue --steps 20 --warmup 5 --cpu-seconds 0) > $OUT/${TAG}_qab_r02_$r.log 2>&1 || { echo "r02 queue failed"; tail -20 $OUT/${TAG}_qab_r02_$r.log; exit 1; }
        timeout -k 10 240 python -u bench.py --workload queue --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/${TAG}_qab_now_$r.log 2>&1 || { echo "queue failed"; tail -20 $OUT/${TAG}_qab_now_$r.log; exit 1; }
        for f in r02 now; do echo "$f $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${TAG}_qab_${f}_$r.log | head -1) $(grep -o '"fold": [0-9.]*' $OUT/${TAG}_qab_${f}_$r.log | head -1)"; done
    done
fi
if [ "$PART" = treeab ]; then
    # the same box: round 3's final tree (tools/r03tree, git worktree of 3227af5, built here)
    # against this one, alternating, on the driver's schedule (bench lines without the
    # host-buffer and string-directory legs)
    for r in $(seq 1 ${ROUNDS:-2}); do
        for W in ${WLS:-uniform zipf}; do
            (cd tools/r03tree && timeout -k 10 240 python -u bench.py --workload $W --steps 20 --warmup 5 --cpu-seconds 0 --no-host-buffer --no-strdir) > $OUT/${TAG}_tab_r03_${W}_$r.log 2>&1 || { echo "r03 $W failed"; tail -20 $OUT/${TAG}_tab_r03_${W}_$r.log; exit 1; }
            timeout -k 10 240 python -u bench.py --workload $W --steps 20 --warmup 5 --cpu-seconds 0 --no-host-buffer --no-strdir --no-sparse > $OUT/${TAG}_tab_now_${W}_$r.log 2>&1 || { echo "now $W failed"; tail -20 $OUT/${TAG}_tab_now_${W}_$r.log; exit 1; }
            for f in r03 now; do echo "$W $f $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/${TAG}_tab_${f}_${W}_$r.log | head -1)"; done
        done
    done
fi
if [ "$PART" = ablate ]; then
    # variants prebuilt here: ABLATE_SET=r04 python tools/ablate.py --build
    ABLATE_SET=${ABLATE_SET:-r04} timeout -k 10 ${ABLATE_TIMEOUT:-900} python -u tools/ablate.py --run --rounds ${ROUNDS:-2} --steps ${STEPS:-5} > $OUT/${TAG}_ablate.log 2>&1
    rc=$?
    cut -c 1-400 $OUT/${TAG}_ablate.log | tail -40
    exit $rc
fi
