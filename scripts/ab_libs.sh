#!/bin/bash
# A/B of in-tree library builds (NLOT_LIB) on the step_trace workload; each result is compared bitwise with the
# reference statuses / iterations / costs.  Usage: scripts/ab_libs.sh OUTDIR lib1.so lib2.so ...
set -e
out=$1
shift
mkdir -p $out
for lib in "$@"; do
    d=$out/${lib%.so}
    NLOT_LIB=$lib timeout -k 10 200 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1
    echo "$lib: $(grep 'traj/s' $d.log)"
    python3 scripts/cmp_res.py profiles/r03/ref/res_t2_B32768_G2.npz $d/res.npz
done
