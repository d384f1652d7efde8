#!/bin/bash
# A/B of the line-search speculation knobs on the metric run (one timed solve each).
set -o pipefail
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > $OUT/base.json 2> $OUT/base.err || exit $?
NLOT_SPEC_BULK=2 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > $OUT/bulk2.json 2> $OUT/bulk2.err || exit $?
NLOT_SPEC_THRESHOLD=2048 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > $OUT/thr2048.json 2> $OUT/thr2048.err || exit $?
NLOT_SPEC_THRESHOLD=32768 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > $OUT/thr32768.json 2> $OUT/thr32768.err || exit $?
