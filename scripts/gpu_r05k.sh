#!/bin/bash
# k_ric phase times (NLOT_RIC_PROF tuning builds: backward / F1 / F2 / F3 + multipliers per solve, summed over the
# groups) for the Newton solves, the corrections and the restoration solves, with the two correction substitutions;
# one batch of 32,768 metric instances through 32,768 slots.
OUT=gpurun_out/r05k
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5profseq r5profpar; do
  NLOT_LIB=libnlot_$v.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 1 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
  grep ric_prof $OUT/$v.log | tail -3
done
