#!/bin/bash
# Restoration solves under k_ric's attempt cap (their inertia correction continues in the next step, as the main
# solves' do): A/B NLOT_RESTO_TRIES=1 (new default) vs 0, bitwise compared; then the solver / restoration GPU tests and smoke
OUT=gpurun_out/r05ar
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in 0 1; do
    NLOT_RESTO_TRIES=$t timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/t$t$rep > $OUT/t$t$rep.log 2>&1 || exit $?
    echo "resto_tries $t rep $rep: $(grep 'traj/s' $OUT/t$t$rep.log)"
  done
done
python3 - <<'PY'
import numpy as np
o = "gpurun_out/r05ar"
a = np.load(f"{o}/t01/res.npz")
for v in ("t11", "t12", "t13", "t02"):
    b = np.load(f"{o}/{v}/res.npz")
    print(v, "bitwise equal to t01:", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "cost")))
PY
timeout -k 10 400 python -u -m pytest tests/test_solver_gpu.py tests/test_resto_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-100
