#!/bin/bash
# Round 4: NLOT_EARLY_VALUE at the bench's scheduling (131,072 instances through 65,536 slots), twice each
OUT=gpurun_out/r04q
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/ab_env.sh $OUT/ab 32768 4 65536 - "NLOT_EARLY_VALUE=1" - "NLOT_EARLY_VALUE=1"
