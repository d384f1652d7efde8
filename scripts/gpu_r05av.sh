#!/bin/bash
OUT=gpurun_out/r05av
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
timeout -k 10 300 python -u scripts/resto_cap_check.py > $OUT/check.log 2>&1; rc=$?
tail -8 $OUT/check.log; exit $rc
