#!/bin/bash
# Round 5: k_ric without scratch (Q_vv / Q_xv, the hg column and P read from LDS where they are used:
# libnlot_r5nospill.so) against the committed tree (libnlot_r5base.so), unicycle_2nd tuning builds, step_trace workload
# (2 x 32,768 metric instances through 32,768 slots), results compared bitwise; both again (run-to-run noise)
OUT=gpurun_out/r05d
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in r5base r5nospill r5base2 r5nospill2; do
  d=$OUT/$v
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
  if [ $v != r5base ]; then python3 scripts/cmp_res.py $OUT/r5base/res.npz $d/res.npz || true; fi
done
