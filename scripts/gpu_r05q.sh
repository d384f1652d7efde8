#!/bin/bash
# When each launch of the bulk's global step starts and ends (scripts/timeline.py offsets), current k_ric
# (libnlot_r5new.so); step_trace workload, one batch of 32,768.
OUT=gpurun_out/r05q
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
NLOT_LIB=libnlot_r5new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/step_trace.py run 32768 1 32768 $GRAFT_REPO_ROOT/$OUT/traced > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $T --out $OUT/timeline.json
gzip -c $T > $OUT/kernel_trace.csv.gz
rm -f $T
