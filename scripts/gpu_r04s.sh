#!/bin/bash
# Round 4: speculation threshold A/B at the bench's scheduling (131,072 instances through 65,536 slots)
OUT=gpurun_out/r04s
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/ab_env.sh $OUT/ab 32768 4 65536 - "NLOT_SPEC_THRESHOLD=16384" "NLOT_SPEC_THRESHOLD=4096" "NLOT_SPEC_BULK=3"
