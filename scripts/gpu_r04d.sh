#!/bin/bash
# Round 4: (1) the test that faulted in r04b/r04c (b5 ackermann_2nd RK4 iterates, restoration line search) alone,
# on the build with default-priority side streams; (2) the whole -m gpu suite; (3) a kernel trace of the opt-in
# thread-per-instance Newton solve (NLOT_RIC_TPI=1) on the step_trace workload.
OUT=gpurun_out/r04d
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v -s -x --timeout 120 --timeout-method thread \
    -k "b5_ackermann2nd_rk4" > $OUT/tests_rk4.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests_rk4.log; tail -3 $OUT/tests_rk4.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -5 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
(cd /tmp && NLOT_RIC_TPI=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/trace_tpi" -o trace \
    -- python3 "$GRAFT_REPO_ROOT/scripts/step_trace.py" run 32768 2 32768 "$GRAFT_REPO_ROOT/$OUT/steps_tpi" \
    > "$GRAFT_REPO_ROOT/$OUT/trace_tpi_run.log" 2>&1) || exit $?
find $OUT/trace_tpi -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_tpi.csv \;
tr=$(find $OUT/trace_tpi -name "*kernel_trace.csv" | head -1)
python3 scripts/step_trace.py reduce "$tr" $OUT/steps_tpi > $OUT/reduce_tpi.log 2>&1
python3 scripts/step_trace.py report $OUT/steps_tpi > $OUT/report_tpi.txt 2>&1; tail -12 $OUT/report_tpi.txt
rm -rf $OUT/trace_tpi
