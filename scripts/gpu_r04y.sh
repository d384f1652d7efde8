#!/bin/bash
# Round 4: k_accept's iterate update with chunked loads (libnlot_wacc.so) against the committed tree (libnlot_wbase.so),
# and with k_iter_b's sigma combination chunked too (libnlot_waccb.so), unicycle_2nd tuning builds, step_trace
# workload, results compared bitwise; base and the last variant again (run-to-run noise)
OUT=gpurun_out/r04y
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in base acc accb base2 accb2; do
  d=$OUT/$v
  NLOT_LIB=libnlot_w${v%2}.so timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
  if [ $v != base ]; then python3 scripts/cmp_res.py $OUT/base/res.npz $d/res.npz || true; fi
done
