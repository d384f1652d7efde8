#!/bin/bash
# A/B of environment knobs on the step_trace workload.  Usage: scripts/ab_env.sh OUTDIR B G SLOTS "ENV=.. ENV=.." ...
# (one quoted assignment list per variant, "-" for none); each result is compared bitwise with the first variant's.
set -e
out=$1; B=$2; G=$3; S=$4
shift 4
mkdir -p $out
i=0
for cfg in "$@"; do
    d=$out/v$i
    if [ "$cfg" = "-" ]; then cfg=""; fi
    env $cfg timeout -k 10 300 python3 scripts/step_trace.py run $B $G $S $d > $d.log 2>&1
    echo "[$cfg] $(grep 'traj/s' $d.log)"
    if [ $i -gt 0 ]; then python3 scripts/cmp_res.py $out/v0/res.npz $d/res.npz || true; fi
    i=$((i + 1))
done
