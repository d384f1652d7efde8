#!/bin/bash
# r02v: k_ric pivot permutations as selects instead of 0/1 blends (libnlot_sel.so): iterate parity on it, then
# A/B bench lines (default K = 4 continuous; 1 run each) against the default build.
OUT=gpurun_out/r02v
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
NLOT_LIB=libnlot_sel.so timeout -k 10 600 python -u -m pytest tests/test_branches_gpu.py tests/test_solver_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/sel_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/sel_tests.log; tail -3 $OUT/sel_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --cpu-sample 0 > $OUT/base.json 2> $OUT/base.err || exit $?
NLOT_LIB=libnlot_sel.so timeout -k 10 400 python -u bench.py --cpu-sample 0 > $OUT/sel.json 2> $OUT/sel.err || exit $?
for f in base sel; do python -c "import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],1), d['config']['status_counts_rank0'], round(d['roofline']['avg_launch_ms'],4))"; done
