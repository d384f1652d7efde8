#!/bin/bash
# Round 4: stream-layout knobs re-measured with the round-4 MLP kernels (statuses compared bitwise)
OUT=gpurun_out/r04p
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/ab_env.sh $OUT/ab 32768 2 32768 - "NLOT_EARLY_VALUE=1" "NLOT_SOC_FORK=1" "NLOT_SOC_FORK=2" "NLOT_SETPRIO=1"
