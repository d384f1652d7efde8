#!/bin/bash
# Second-order corrections as a parallel-over-knots substitution with a short chain (libnlot_r5socpar.so) against
# the stage-by-stage sweep (r5socseq, NLOT_SOC_SEQ), unicycle_2nd tuning builds, step_trace workload (2 x 32,768
# metric instances through 32,768 slots); then a kernel trace of the new build for the step's critical path.
OUT=gpurun_out/r05i
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in r5socseq r5socpar r5socseq2 r5socpar2; do
  d=$OUT/$v
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $d.log)"
done
python3 -c "
import numpy as np
for v in ('r5socseq','r5socpar','r5socseq2','r5socpar2'):
    a=np.load('$OUT/'+v+'/res.npz'); print(v, np.bincount(a['status'],minlength=7).tolist(), 'iters', int(a['iters'].sum()), 'wall', float(a['wall']))
"
python3 scripts/cmp_res.py $OUT/r5socseq/res.npz $OUT/r5socseq2/res.npz || true
python3 scripts/cmp_res.py $OUT/r5socpar/res.npz $OUT/r5socpar2/res.npz || true
cd /tmp || exit 1
NLOT_LIB=libnlot_r5socpar.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/step_trace.py run 32768 1 32768 $GRAFT_REPO_ROOT/$OUT/traced > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $T --out $OUT/timeline.json
python3 scripts/step_trace.py reduce $T $OUT/traced > $OUT/reduce.log 2>&1
python3 scripts/step_trace.py report $OUT/traced > $OUT/report.txt 2>&1
rm -f $T
