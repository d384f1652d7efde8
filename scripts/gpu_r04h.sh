#!/bin/bash
# Round 4: K concurrent solver calls (own stream + workspace each) against one call on the same 65,536 seeded
# metric instances (results compared bitwise).
OUT=gpurun_out/r04h
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for K in 2 4; do
  timeout -k 10 300 python3 -u scripts/concurrent_solve.py 32768 2 32768 $K > $OUT/conc_K${K}.log 2>&1 || exit $?
  tail -1 $OUT/conc_K${K}.log
done
