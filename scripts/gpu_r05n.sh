#!/bin/bash
# Scheduling knobs with the current k_ric (libnlot_r5new.so), the corrections' chain being the step's critical path
# (scripts/timeline.py: it ends 1.1 ms after the Newton solves): early value launch off, the correction stream at
# the highest priority, side-stream waves at raised issue priority; step_trace workload (2 x 32,768).
OUT=gpurun_out/r05n
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
run() {  # name, env assignments...
  local n=$1; shift
  env "$@" NLOT_LIB=libnlot_r5new.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$n > $OUT/$n.log 2>&1 || exit $?
  echo "$n: $(grep 'traj/s' $OUT/$n.log)"
}
run base X=0
run ev0 NLOT_EARLY_VALUE=0
run prio2 NLOT_STREAM_PRIO=2
run setprio NLOT_SETPRIO=1
run prio2_setprio NLOT_STREAM_PRIO=2 NLOT_SETPRIO=1
run base2 X=0
