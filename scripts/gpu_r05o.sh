#!/bin/bash
# k_ric occupancy: 3 waves per SIMD for the Newton solve (ric3: 168 VGPRs, 476 B/lane scratch), for the corrections
# (soc3: 332 B), both, against 2 (r5new); step_trace workload (2 x 32,768).
OUT=gpurun_out/r05o
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5new r5ric3 r5soc3 r5both3 r5new2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
