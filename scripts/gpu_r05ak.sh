#!/bin/bash
# sampled event timing (one step in 8, rotating position) against every step: per-launch averages must agree
OUT=gpurun_out/r05ak
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for e in 8 1; do
  NLOT_BENCH_TIMING_EVERY=$e timeout -k 10 300 python -u bench.py --gpus 1 --steps 8 --warmup 2 --cpu-sample 0 > $OUT/bench_e$e.json 2> $OUT/bench_e$e.err || exit $?
  python -c "
import json; d=json.load(open('$OUT/bench_e$e.json'))
print('every $e', round(d['value'],1), [(k, round(d[k]['avg_launch_ms'],4), round(d[k]['frac'],4), d[k].get('timed_launches')) for k in ('roofline','roofline_mlp_full','roofline_mlp_value')], {k: round(d['config'][k],1) for k in ('solver_step_kernel_ms_per_step','ric_ms_per_step','mlp_ms_per_step')})"
done
