#!/bin/bash
# A/B: NLOT_JOIN_V1=1 (the restoration stream joins the early value launch; one cross-stream wait before the second
# value launch) vs 0; results compared bitwise
OUT=gpurun_out/r05an
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for rep in 1 2 3; do
  for j in 0 1; do
    NLOT_JOIN_V1=$j timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/j$j$rep > $OUT/j$j$rep.log 2>&1 || exit $?
    echo "join $j rep $rep: $(grep 'traj/s' $OUT/j$j$rep.log)"
  done
done
python3 - <<'PY'
import numpy as np
o = "gpurun_out/r05an"
a = np.load(f"{o}/j01/res.npz")
for v in ("j11", "j12", "j02"):
    b = np.load(f"{o}/{v}/res.npz")
    print(v, "bitwise equal to j01:", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "cost")))
PY
