#!/bin/bash
# r02p: speculation-threshold A/B on the metric workload (env knobs, same build; 1 timed solve each), then
# refreshed stress and b6 bench lines with kernel-trace stats of the stress run.
OUT=gpurun_out/r02p
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --steps 1 --warmup 1 --cpu-sample 0"
for t in 2048 8192 32768; do
  NLOT_SPEC_THRESHOLD=$t timeout -k 10 300 $B > $OUT/spec$t.json 2> $OUT/spec$t.err || exit $?
done
NLOT_SPEC_BULK=2 timeout -k 10 300 $B > $OUT/bulk2.json 2> $OUT/bulk2.err || exit $?
for f in spec2048 spec8192 spec32768 bulk2; do python -c "import json,sys; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['config']['status_counts_rank0'], d['config']['lockstep_global_steps'], round(d['ms_per_step'],1), round(d['roofline_mlp_value']['avg_launch_ms'],4))"; done
timeout -k 10 600 python -u bench.py --workload stress --steps 1 --warmup 1 > $OUT/stress.json 2> $OUT/stress.err || exit $?
tail -c 600 $OUT/stress.json
timeout -k 10 600 python -u bench.py --workload b6 --steps 1 --warmup 1 > $OUT/b6.json 2> $OUT/b6.err || exit $?
tail -c 600 $OUT/b6.json
