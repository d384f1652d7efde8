#!/bin/bash
# Round 4: the split-parity tests and smoke on the fixture with final-iterate reproducibility.
OUT=gpurun_out/r04i
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_solver_gpu.py tests/test_b6_gpu.py tests/test_resto_gpu.py -m gpu -v -s \
    --timeout 300 --timeout-method thread -k "batch or full_solves or statuses_on_metric" > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log; grep "^\[parity\]" $OUT/tests.log | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-300
