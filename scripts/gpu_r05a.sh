#!/bin/bash
# Round 5: iterate parity of the constraint-row bounds (general_bounds, the reference's NLP form) against the oracle,
# and of the variable-bound form, on every branch, the learned SDF, the restoration cases and b6.
OUT=gpurun_out/r05a
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread \
    tests/test_branches_gpu.py::test_iterates_match_oracle tests/test_solver_gpu.py::test_iterates_match_oracle_b2 \
    tests/test_solver_gpu.py::test_iterates_match_oracle_learned tests/test_resto_gpu.py::test_restoration_iterates_match_oracle \
    tests/test_b6_gpu.py::test_b6_iterates_match_oracle tests/test_solver_gpu.py::test_tiny_step_rule_matches_oracle \
    tests/test_solver_gpu.py::test_safeguards_iterate_parity > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
grep -E "PASSED|FAILED|ERROR" $OUT/tests.log | cut -c1-200 | tail -80
exit $rc
