#!/bin/bash
# Final tree (k_step_end, sampled event timing): the new GPU tests, rocprofv3 --kernel-trace --stats over the driver's
# bench command (per-kernel averages against the bench's sampled hipEvent averages), smoke
OUT=gpurun_out/r05ao
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_solver_gpu.py -m gpu -q -k "sampled or knobs" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 800 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 \
    > "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.err")
rc=$?
find $OUT/prof -name "*kernel_trace.csv" -delete
echo "rocprof exit $rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/rocprof_fracs.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/bench_rocprof.json $OUT/mlp_dispatch_fracs_r05ao.json | tail -8
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-120
