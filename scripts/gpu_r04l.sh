#!/bin/bash
# Round 4: branch full-solve split-parity tests after restoring the round-3 knot evaluation
OUT=gpurun_out/r04l
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_branches_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
    -k "full_solves" > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -2 $OUT/tests.log; grep "trapezoid gpu\|polygon gpu" $OUT/tests.log | cut -c1-200
