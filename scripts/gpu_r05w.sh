#!/bin/bash
# k_iter_b with its reads ahead of its writes (libnlot_r5itb.so: theta / phi's passes loaded together, the knot's step
# recovery inputs before its first store, the controls' bound rows in chunks) against the committed tree (r5preA);
# step_trace workload (2 x 32,768), bitwise comparison.
OUT=gpurun_out/r05w
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5preA r5itb r5preA2 r5itb2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5preA/res.npz $OUT/r5itb/res.npz || true
