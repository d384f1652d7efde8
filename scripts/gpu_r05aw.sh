#!/bin/bash
# k_ric<DYN, true> over the whole restoration list (was clamped to the host's stale grid bound): benchmark 6 with and
# without the restoration attempt cap (statuses must now agree), then the b6 / restoration / solver GPU tests
OUT=gpurun_out/r05aw
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
for t in 1 0; do
  NLOT_RESTO_TRIES=$t timeout -k 10 400 python -u bench.py --gpus 1 --workload b6 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/b6_t$t.json 2> $OUT/b6_t$t.err || exit $?
  python -c "import json; d=json.load(open('$OUT/b6_t$t.json')); print('b6 resto_tries $t', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'])"
done
timeout -k 10 500 python -u -m pytest tests/test_b6_gpu.py tests/test_resto_gpu.py tests/test_solver_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; exit $rc
