#!/bin/bash
# Final tree: the driver's bench command, the same with the CPU baseline after the timed region (--cpu-overlap off,
# ADVICE r04), and the variable-bound form
OUT=gpurun_out/r05ab
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); print('default', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-overlap off > $OUT/bench_overlap_off.json 2> $OUT/bench_overlap_off.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_overlap_off.json')); print('overlap off', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --bounds variable --cpu-sample 0 > $OUT/bench_varbounds.json 2> $OUT/bench_varbounds.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_varbounds.json')); print('varbounds', d['value'], d['config']['status_counts_rank0'])"
