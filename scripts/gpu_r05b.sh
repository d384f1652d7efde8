#!/bin/bash
# Round 5: the two rows-form test fixes, then the driver's bench command in the reference's NLP form (constraint-row
# bounds, the default) and with variable bounds (the figures reported beside it).
OUT=gpurun_out/r05b
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread \
    tests/test_solver_gpu.py::test_iterates_match_oracle_b2 tests/test_solver_gpu.py::test_tiny_step_rule_matches_oracle \
    > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_rows.json 2> $OUT/bench_rows.err || exit $?
tail -c 600 $OUT/bench_rows.json
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --bounds variable --cpu-sample 0 > $OUT/bench_var.json 2> $OUT/bench_var.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_var.json')); print(d['value'], d['config']['status_counts_rank0'])"
