#!/bin/bash
# Default attempt cap at every batch size (ric_tries_min 0): metric A/B reps against the old threshold, the GPU suite, smoke
OUT=gpurun_out/r05ba
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for m in 2048 0; do
    NLOT_RIC_TRIES_MIN=$m timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/m$m$rep > $OUT/m$m$rep.log 2>&1 || exit $?
    echo "tries_min $m rep $rep: $(grep 'traj/s' $OUT/m$m$rep.log)"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-100
