#!/bin/bash
# k_iter_a at 3 waves per SIMD (libnlot_r5a3.so: 168 VGPRs, 856 B/lane scratch) against 2 (r5itb: 256, 536 B)
OUT=gpurun_out/r05af
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5itb r5a3 r5itb2 r5a32; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
