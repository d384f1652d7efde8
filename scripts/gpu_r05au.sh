#!/bin/bash
# Benchmark 6 (restoration-heavy) with and without the restoration attempt cap, same box; statuses must agree
OUT=gpurun_out/r05au
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for t in 1 0; do
  NLOT_RESTO_TRIES=$t timeout -k 10 400 python -u bench.py --gpus 1 --workload b6 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/b6_t$t.json 2> $OUT/b6_t$t.err || exit $?
  python -c "import json; d=json.load(open('$OUT/b6_t$t.json')); print('b6 resto_tries $t', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'])"
done
