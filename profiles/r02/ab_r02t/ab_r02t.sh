#!/bin/bash
# r02t: continuous-batching A/B on the metric workload (no CPU baseline): slots = batch vs all at once, K = 2 and 4.
OUT=gpurun_out/r02t
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
B="python -u bench.py --cpu-sample 0 --warmup 1"
timeout -k 10 400 $B --steps 2 --slots 131072 > $OUT/k2_all.json 2> $OUT/k2_all.err || exit $?
timeout -k 10 400 $B --steps 4 > $OUT/k4_cont.json 2> $OUT/k4_cont.err || exit $?
timeout -k 10 400 $B --steps 4 --slots 131072 > $OUT/k4_s131k.json 2> $OUT/k4_s131k.err || exit $?
for f in k2_all k4_cont k4_s131k; do python -c "import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],1), d['config']['scheduling'][:120])"; done
