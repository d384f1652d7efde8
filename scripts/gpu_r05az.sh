#!/bin/bash
# A/B: the attempt cap in the tail too (NLOT_RIC_TRIES_MIN=0) vs only while > 2048 instances are active (default);
# metric step-trace workload and benchmark 6
OUT=gpurun_out/r05az
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for m in 2048 0; do
  NLOT_RIC_TRIES_MIN=$m timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/m$m > $OUT/m$m.log 2>&1 || exit $?
  echo "tries_min $m metric: $(grep 'traj/s' $OUT/m$m.log)"
done
for m in 2048 0; do
  NLOT_RIC_TRIES_MIN=$m timeout -k 10 400 python -u bench.py --gpus 1 --workload b6 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/b6_m$m.json 2> $OUT/b6_m$m.err || exit $?
  python -c "import json; d=json.load(open('$OUT/b6_m$m.json')); print('tries_min $m b6', d['value'], d['config']['status_counts_rank0'])"
done
