#!/bin/bash
# k_ric's per-stage HBM stores deferred by one stage (libnlot_r5flush.so: from LDS after the next stage's ring wait)
# against the committed tree (r5itb); bitwise comparison; k_ric phase profiles of both.
OUT=gpurun_out/r05ad
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5itb r5flush r5itb2 r5flush2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5itb/res.npz $OUT/r5flush/res.npz || true
for v in r5itbprof r5flushprof; do
  NLOT_LIB=libnlot_$v.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 1 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v"; grep ric_prof $OUT/$v.log | tail -3
done
