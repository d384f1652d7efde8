#!/bin/bash
# A/B on the round-end tree: the correction chain forked after the full MLP launch (NLOT_SOC_FORK=2) vs after k_iter_a
# (0, default); results compared bitwise
OUT=gpurun_out/r05at
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for rep in 1 2 3; do
  for f in 0 2; do
    NLOT_SOC_FORK=$f timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/f$f$rep > $OUT/f$f$rep.log 2>&1 || exit $?
    echo "soc_fork $f rep $rep: $(grep 'traj/s' $OUT/f$f$rep.log)"
  done
done
python3 - <<'PY'
import numpy as np
o = "gpurun_out/r05at"
a = np.load(f"{o}/f01/res.npz")
for v in ("f21", "f22", "f23"):
    b = np.load(f"{o}/{v}/res.npz")
    print(v, "bitwise equal to f01:", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "cost")))
PY
