#!/bin/bash
# Pinned iterates with both nets, b6 batch with both nets, metric batch with both nets, the branch full solves.
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -s \
  tests/test_pinned_iterates_gpu.py tests/test_b6_gpu.py tests/test_branches_gpu.py \
  "tests/test_solver_gpu.py::test_batch_learned_sdf_matches_oracle[rows]" -k "not varbounds" > $OUT/tests.log 2>&1
rc=$?
grep -E "^\[pinned\]|^\[parity\]|excused|PASS|FAIL|passed|failed" $OUT/tests.log | cut -c1-400
echo "exit $rc"
