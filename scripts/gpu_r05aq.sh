#!/bin/bash
# A/B: NLOT_STREAM_PRIO=1 (restoration stream at the highest priority; its chain ends after k_iter_b in ~15 % of the
# bulk steps, timeline_r05al) vs default streams; results compared bitwise
OUT=gpurun_out/r05aq
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for rep in 1 2 3; do
  for pr in 0 1; do
    NLOT_STREAM_PRIO=$pr timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/p$pr$rep > $OUT/p$pr$rep.log 2>&1 || exit $?
    echo "prio $pr rep $rep: $(grep 'traj/s' $OUT/p$pr$rep.log)"
  done
done
python3 - <<'PY'
import numpy as np
o = "gpurun_out/r05aq"
a = np.load(f"{o}/p01/res.npz")
for v in ("p11", "p12", "p13"):
    b = np.load(f"{o}/{v}/res.npz")
    print(v, "bitwise equal to p01:", all(np.array_equal(a[k], b[k]) for k in ("status", "iters", "cost")))
PY
