#!/bin/bash
# Round 5, final tree: smoke and the driver's bench command as the driver runs them (bench defaults: CPU baseline
# after the timed region)
OUT=gpurun_out/r05ag
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-160
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'], d['cpu_baseline']['value'], d['roofline']['frac'])"
