#!/bin/bash
# Round 4: the restoration kernels' occupancy (NLOT_WPE_RA / RLS / RRIC: few wavefronts, latency counts), unicycle_2nd
# tuning builds (libnlot_w*.so), step_trace workload; every variant compared bitwise with the base build
OUT=gpurun_out/r04v
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in base ra1 rr1 all1; do
  d=$OUT/$v
  NLOT_LIB=libnlot_w$v.so timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
  if [ $v != base ]; then python3 scripts/cmp_res.py $OUT/base/res.npz $d/res.npz || true; fi
done
