#!/bin/bash
# Round 4: the split-parity tests on the six-run fixture (metric 128, b6 24, b2, restoration full solves), smoke,
# then the solver SQ PMC passes.
OUT=gpurun_out/r04g
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_solver_gpu.py tests/test_b6_gpu.py tests/test_resto_gpu.py -m gpu -v -s \
    --timeout 300 --timeout-method thread -k "batch or full_solves or statuses_on_metric" > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log; grep "\[parity\]" $OUT/tests.log | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log | cut -c1-300
timeout -k 10 600 python -u scripts/debug_fixture_divergence.py b6 5 --ks 5,10,20,40,80,160,320,1000 > $OUT/div_b6_5.log 2>&1 || exit $?
cat $OUT/div_b6_5.log | cut -c1-250
OUT_TAG=r04sq bash scripts/pmc_solver_sq.sh
