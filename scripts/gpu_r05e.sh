#!/bin/bash
# Round 5: the restoration chain (k_resto_a included) on its own stream, forked after the full MLP launch, with the
# round-4 k_ric (libnlot_r5vara.so), with Q_vv / Q_xv read from LDS (r5varb: 88 B/lane scratch instead of 196) and
# with the scratch-free k_ric (r5resto), against the committed tree (r5base); unicycle_2nd tuning builds, step_trace
# workload (2 x 32,768 metric instances through 32,768 slots), results compared with the base
OUT=gpurun_out/r05e
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in r5base r5vara r5varb r5resto r5base2 r5vara2; do
  d=$OUT/$v
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
  if [ $v != r5base ]; then python3 scripts/cmp_res.py $OUT/r5base/res.npz $d/res.npz || true; fi
done
