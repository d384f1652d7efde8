#!/bin/bash
# k_accept's line-search trials with the residual-store flag a compile-time constant (libnlot_r5trial.so) against the
# committed tree (r5itb); step_trace workload (2 x 32,768), bitwise comparison.
OUT=gpurun_out/r05x
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5itb r5trial r5itb2 r5trial2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5itb/res.npz $OUT/r5trial/res.npz || true
