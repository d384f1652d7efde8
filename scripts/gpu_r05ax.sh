#!/bin/bash
# Final tree (restoration list fix): the whole GPU suite, smoke, and the driver's bench command
OUT=gpurun_out/r05ax
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -1 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log | cut -c1-100
timeout -k 10 420 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'], d['cpu_baseline']['value'], r['frac'], r['avg_launch_ms'])"
