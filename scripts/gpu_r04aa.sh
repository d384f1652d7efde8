#!/bin/bash
# Round 4: k_iter_a's lane-strided sums (theta/phi, optimality error, complementarity) through chunked_update
# (libnlot_wia.so) against the committed tree (libnlot_wbase.so), unicycle_2nd tuning builds, step_trace workload,
# results compared bitwise; both twice (run-to-run noise)
OUT=gpurun_out/r04aa
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in base ia base2 ia2; do
  d=$OUT/$v
  NLOT_LIB=libnlot_w${v%2}.so timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
  if [ $v != base ]; then python3 scripts/cmp_res.py $OUT/base/res.npz $d/res.npz || true; fi
done
