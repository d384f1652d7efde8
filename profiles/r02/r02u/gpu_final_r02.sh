#!/bin/bash
# Final r02 check: the whole -m gpu suite, smoke(), the default bench line (with the CPU baseline), and a
# kernel-trace summary of the default bench.
OUT=gpurun_out/r02u
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/gpu_tests.log; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-200
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -c 1200 $OUT/bench.json
(cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-sample 0 --warmup 0 \
    > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2>&1)
