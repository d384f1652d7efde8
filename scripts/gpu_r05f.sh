#!/bin/bash
# Round 5: the GPU suite on the reference's NLP form (the variable-bound batch test waits for its fixture), smoke, and
# the driver's bench command, on the tree with the restoration chain on its own stream
OUT=gpurun_out/r05f
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -k "not varbounds" \
    > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log; grep -E "^\[parity\]|^\[pinned\]" $OUT/tests.log | cut -c1-250
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log | cut -c1-300
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['config']['status_counts_rank0'])"
