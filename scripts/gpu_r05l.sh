#!/bin/bash
# k_ric's forward passes with every row of a knot loaded before the first store (F1: closed-loop maps; F3 and the
# multipliers: both right-hand sides per knot) and the correction sweep prefetching three stages (libnlot_r5new.so)
# against the committed sweep (r5socseq); bitwise comparison, then the phase profile of the new build.
OUT=gpurun_out/r05l
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5socseq r5new r5socseq2 r5new2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5socseq/res.npz $OUT/r5new/res.npz || true
NLOT_LIB=libnlot_r5newprof.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 1 32768 $OUT/prof > $OUT/prof.log 2>&1 || exit $?
grep ric_prof $OUT/prof.log | tail -3
