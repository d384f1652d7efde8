#!/bin/bash
# Where the main stream waits for the side streams (NLOT_WAIT_LATE 0 / 1 / 2, libnlot_r5wait.so): the trace put a
# 64 us gap between k_iter_b and the second value launch; step_trace workload (2 x 32,768), bitwise comparison.
OUT=gpurun_out/r05aa
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for w in 0 1 2 0b 1b 2b; do
  NLOT_WAIT_LATE=${w%b} NLOT_LIB=libnlot_r5wait.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/w$w > $OUT/w$w.log 2>&1 || exit $?
  echo "wait_late $w: $(grep 'traj/s' $OUT/w$w.log)"
done
python3 scripts/cmp_res.py $OUT/w0/res.npz $OUT/w1/res.npz || true
python3 scripts/cmp_res.py $OUT/w0/res.npz $OUT/w2/res.npz || true
