#!/bin/bash
# Round-end lines of BASELINE's other GPU configurations: benchmark 6 (configs[3]) and stress (configs[4]), defaults
OUT=gpurun_out/r05ay
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --gpus 1 --workload b6 > $OUT/bench_b6.json 2> $OUT/bench_b6.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_b6.json')); print('b6', d['value'], d['config']['status_counts_rank0'])"
timeout -k 10 500 python -u bench.py --gpus 1 --workload stress > $OUT/bench_stress.json 2> $OUT/bench_stress.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_stress.json')); print('stress', d['value'], d['config']['status_counts_rank0'])"
