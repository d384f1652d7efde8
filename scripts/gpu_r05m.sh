#!/bin/bash
# Phase profile of k_iter_a / k_iter_b / k_accept (NLOT_KPROF tuning build) and the step's critical path from a
# kernel trace of the current k_ric (libnlot_r5new.so); step_trace workload, one batch of 32,768.
OUT=gpurun_out/r05m
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
NLOT_LIB=libnlot_r5kprof.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 1 32768 $OUT/kprof > $OUT/kprof.log 2>&1 || exit $?
grep -E "kprof|traj/s" $OUT/kprof.log | tail -4
cd /tmp || exit 1
NLOT_LIB=libnlot_r5new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/step_trace.py run 32768 1 32768 $GRAFT_REPO_ROOT/$OUT/traced > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $T --out $OUT/timeline.json
python3 scripts/timeline.py $T --min-active 1 --out $OUT/timeline_all.json > /dev/null
rm -f $T
