#!/bin/bash
# One-corner knot evaluation (libnlot_r5onec.so: no per-corner arrays; k_iter_a scratch 536 -> 288 B/lane, k_accept
# 304 -> 288, k_resto_a 656 -> 204) against the committed tree (r5preA); step_trace workload (2 x 32,768), bitwise
# comparison.
OUT=gpurun_out/r05v
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in r5preA r5onec r5preA2 r5onec2; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5preA/res.npz $OUT/r5onec/res.npz || true
