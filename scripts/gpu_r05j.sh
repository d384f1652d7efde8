#!/bin/bash
# Where the second-order corrections' chain forks (NLOT_SOC_FORK 0: after k_iter_a, the default; 1: at the start of
# the step, before the full MLP launch; 2: after it) x the two correction substitutions (r5socseq: stage-by-stage
# sweep; r5socpar: parallel over knots with a short chain); step_trace workload (2 x 32,768 metric instances).
OUT=gpurun_out/r05j
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for f in 1 2 0; do
  for v in r5socseq r5socpar; do
    d=$OUT/${v}_f$f
    NLOT_SOC_FORK=$f NLOT_LIB=libnlot_$v.so timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
    echo "$v fork $f: $(grep 'traj/s' $d.log)"
  done
done
