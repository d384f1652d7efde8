#!/bin/bash
# Round 4, first GPU call: a test subset on the new build (ABI v11, 1024-entry filters), then an A/B of the
# side-stream priority knobs on 2 seeded metric batches of 32,768 through 32,768 slots (statuses compared bitwise).
OUT=gpurun_out/r04a
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
    -k "test_abi or iterates_match_oracle_b2 or continuous_batching or rrt or test_mlp_matches" > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/ab_env.sh $OUT/ab 32768 2 32768 - "NLOT_SETPRIO=1" "NLOT_STREAM_PRIO=1" "NLOT_STREAM_PRIO=2" \
    "NLOT_SETPRIO=1 NLOT_STREAM_PRIO=2"
# per-step anatomy of the default configuration (kernel trace reduced per step)
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/trace" -o trace \
    -- python3 "$GRAFT_REPO_ROOT/scripts/step_trace.py" run 32768 2 32768 "$GRAFT_REPO_ROOT/$OUT/steps" \
    > "$GRAFT_REPO_ROOT/$OUT/trace_run.log" 2>&1) || exit $?
tr=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/step_trace.py reduce "$tr" $OUT/steps > $OUT/reduce.log 2>&1 && \
python3 scripts/step_trace.py report $OUT/steps > $OUT/report.txt 2>&1; tail -40 $OUT/report.txt
rm -f "$tr"
