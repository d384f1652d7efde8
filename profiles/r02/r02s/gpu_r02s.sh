#!/bin/bash
# r02s: continuous batching — its parity test (+ the solver suite), then bench lines with it on (default) and off,
# and a kernel trace of the default bench.
OUT=gpurun_out/r02s
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/solver_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/solver_tests.log; tail -3 $OUT/solver_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $OUT/bench_cont.json 2> $OUT/bench_cont.err || exit $?
timeout -k 10 400 python -u bench.py --cpu-sample 0 --continuous off > $OUT/bench_off.json 2> $OUT/bench_off.err || exit $?
for f in bench_cont bench_off; do python -c "import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['ms_per_step'], d['config']['status_counts_rank0'], d['config']['scheduling'])"; done
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-sample 0 --warmup 0 \
    > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2>&1)
