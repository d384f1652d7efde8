#!/bin/bash
# Round 4: rocprofv3 --kernel-trace --stats over the driver's bench command itself (20 timed batches, 5 warm-up; the
# CPU baseline skipped under the profiler), so the summary's per-kernel averages can be set beside the bench line's
# event-timed ones.  Only the stats are kept (the full trace is deleted: hundreds of thousands of dispatches).
OUT=gpurun_out/r04t
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 \
    > "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.err")
rc=$?
find $OUT/prof -name "*kernel_trace.csv" -delete
echo "rocprof exit $rc"
tail -c 300 $OUT/bench_rocprof.json
exit $rc
