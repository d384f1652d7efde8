#!/bin/bash
# r02o: k_ric with its global stores deferred by one stage (libnlot_defer.so): iterate/batch parity tests on it,
# then A/B bench lines (1 timed solve each) against the default build; smoke() of the default build.
OUT=gpurun_out/r02o
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
NLOT_LIB=libnlot_defer.so timeout -k 10 600 python -u -m pytest tests/test_solver_gpu.py tests/test_branches_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/defer_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/defer_tests.log; tail -3 $OUT/defer_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 1 --warmup 1 --cpu-sample 0"
timeout -k 10 300 $B > $OUT/base.json 2> $OUT/base.err || exit $?
NLOT_LIB=libnlot_defer.so timeout -k 10 300 $B > $OUT/defer.json 2> $OUT/defer.err || exit $?
for f in base defer; do python -c "import json,sys; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['config']['status_counts_rank0'], d['config']['lockstep_global_steps'], round(d['roofline']['avg_launch_ms'],4), round(d['ms_per_step'],1))"; done
timeout -k 10 300 python -u -m pytest tests/test_boundary_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/boundary.log 2>&1; tail -2 $OUT/boundary.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke exit $?"; tail -2 $OUT/smoke.log
