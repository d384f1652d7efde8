#!/bin/bash
# Round 5 final tree, part 2: smoke, the driver's bench command, the b6 bench line (BASELINE configs[3]) and the
# cpu-overlap A/B (the CPU baseline during the warm-up, or after the timed region)
OUT=gpurun_out/r05t
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-200
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'])"
timeout -k 10 600 python -u bench.py --gpus 1 --workload b6 > $OUT/bench_b6.json 2> $OUT/bench_b6.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_b6.json')); print('b6', d['value'], d['config'].get('status_counts_rank0'))"
