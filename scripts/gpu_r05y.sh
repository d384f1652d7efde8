#!/bin/bash
# The b6 batch test (the fixture's WIDE outcomes in the chaotic envelope, binomial sampling slack) and the pinned
# iterates (WIDE-start excusal) on the final tree
OUT=gpurun_out/r05y
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_b6_gpu.py tests/test_pinned_iterates_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
grep -E "^\[parity\] b6|^\[pinned\].*(outside|excused|WIDE)" $OUT/tests.log | cut -c1-300
exit $rc
