#!/bin/bash
# Round 4: thread-per-instance Newton solve (k_ric_tpi) — iterate parity against the oracle on every branch, then an
# A/B against the lane-group k_ric (NLOT_RIC_TPI=0) on 2 seeded metric batches of 32,768 through 32,768 slots.
OUT=gpurun_out/r04b
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread \
    -k "iterates or tiny_step or safeguards or test_abi or continuous_batching_same_results" > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -5 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/ab_env.sh $OUT/ab 32768 2 32768 - "NLOT_RIC_TPI=0"
