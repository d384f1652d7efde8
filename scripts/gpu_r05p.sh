#!/bin/bash
# The corrections' substitution with 8 lanes per instance (libnlot_r5g8.so: 8 instances per wavefront, half the
# waves) against 16 (r5new); step_trace workload (2 x 32,768), bitwise comparison, then the timeline of r5g8.
OUT=gpurun_out/r05p
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for v in r5new r5g8 r5new2 r5g82; do
  NLOT_LIB=libnlot_${v%2}.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$v > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(grep 'traj/s' $OUT/$v.log)"
done
python3 scripts/cmp_res.py $OUT/r5new/res.npz $OUT/r5g8/res.npz || true
cd /tmp || exit 1
NLOT_LIB=libnlot_r5g8.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/step_trace.py run 32768 1 32768 $GRAFT_REPO_ROOT/$OUT/traced > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $T --out $OUT/timeline.json | grep -E "wall|ric|iter|accept|mlp|soc_end"
rm -f $T
