#!/bin/bash
# Round 5 final tree, part 1: the whole GPU suite (both NLP forms, both MLP arithmetics in the parity tests)
OUT=gpurun_out/r05s2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
grep -E "^\[parity\]|^\[pinned\]" $OUT/tests.log | cut -c1-200 | tail -40
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
exit $rc
