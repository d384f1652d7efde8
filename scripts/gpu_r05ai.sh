#!/bin/bash
# A/B: the per-step counter bookkeeping as one kernel (k_step_end) vs the D2H / fill / D2D copies (NLOT_STEP_KERNEL=0),
# each with and without bench.py's hipEvent timing (STEP_TIMING=1); results compared bitwise
OUT=gpurun_out/r05ai
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for rep in 1 2; do
  for v in k1t0 k0t0 k1t1 k0t1; do
    k=${v:1:1}; t=${v:3:1}
    NLOT_STEP_KERNEL=$k STEP_TIMING=$t timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v$rep > $OUT/$v$rep.log 2>&1 || exit $?
    echo "$v rep $rep: $(grep 'traj/s' $OUT/$v$rep.log)"
  done
done
python3 - <<'PY'
import numpy as np
o = "gpurun_out/r05ai"
a = np.load(f"{o}/k0t01/res.npz")
for v in ("k1t01", "k1t11", "k0t11", "k1t02", "k0t02"):
    b = np.load(f"{o}/{v}/res.npz")
    print(v, "status/iters/cost bitwise equal to k0t01:", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "cost")))
PY
