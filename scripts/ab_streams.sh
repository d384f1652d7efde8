#!/bin/bash
# A/B of the step's stream layout (NLOT_SOC_FORK, NLOT_EARLY_VALUE) on the step_trace workload; each result is
# compared bitwise with the reference statuses / iterations / costs.  Usage: scripts/ab_streams.sh OUTDIR
set -e
out=$1
mkdir -p $out
for cfg in "0 0" "1 0" "2 0" "0 1" "2 1"; do
    set -- $cfg
    d=$out/fork$1_early$2
    NLOT_SOC_FORK=$1 NLOT_EARLY_VALUE=$2 timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1
    grep "traj/s" $d.log
    python3 scripts/cmp_res.py profiles/r03/ref/res_t2_B32768_G2.npz $d/res.npz
done
