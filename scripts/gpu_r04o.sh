#!/bin/bash
# Round 4: bulk line-search speculation A/B (candidates per later round in the bulk: 1 / 2 (default) / 3) with the
# round-4 MLP kernels, statuses compared bitwise; then the stress workload's bench line.
OUT=gpurun_out/r04o
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/ab_env.sh $OUT/ab 32768 2 32768 - "NLOT_SPEC_BULK=1" "NLOT_SPEC_BULK=3" || exit $?
timeout -k 10 600 python -u bench.py --workload stress --steps 4 --warmup 1 > $OUT/bench_stress.json \
    2> $OUT/bench_stress.err || exit $?
tail -c 600 $OUT/bench_stress.json
