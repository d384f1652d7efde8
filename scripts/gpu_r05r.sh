#!/bin/bash
# k_iter_a's reductions with their loads issued ahead (Pre): A = the optimality measures' 13 passes, B = A + theta/phi,
# full = B + the primal-dual error and complementarity passes (k_iter_a scratch 536 / 712 / 712 B per lane), against
# r5new; step_trace workload (2 x 32,768), bitwise comparison.
OUT=gpurun_out/r05r
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5new r5preA r5preB r5prefull r5new2 r5preA2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
for v in r5preA r5preB r5prefull; do python3 scripts/cmp_res.py $OUT/r5new/res.npz $OUT/$v/res.npz || true; done
