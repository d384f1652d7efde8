#!/bin/bash
# Final tree: the driver's bench command as the driver runs it (CPU baseline after the timed region)
OUT=gpurun_out/r05bb
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'], d['cpu_baseline']['value'], r['frac'], r['avg_launch_ms'], r['rocprof'])"
