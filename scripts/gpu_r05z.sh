#!/bin/bash
# Where b6 instance 3 (variable-bound form) leaves the oracle's pinned path under both nets
OUT=gpurun_out/r05z
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for a in split_bf16 f32; do
  timeout -k 10 400 python3 -u scripts/pin_probe.py --case b6 --form varbounds --inst 3 --kmin 2 --kmax 87 --kstep 5 --arith $a > $OUT/probe_$a.log 2>&1 || exit $?
done
cat $OUT/probe_*.log | grep -v amdgpu
