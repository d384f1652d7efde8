#!/bin/bash
# MLP kernel tests with both MFMA arithmetics, and the stress bench line (BASELINE configs[4]) on the final tree
OUT=gpurun_out/r05ah
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_mlp_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/mlp_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" $OUT/mlp_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --gpus 1 --workload stress > $OUT/bench_stress.json 2> $OUT/bench_stress.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_stress.json')); print('stress', d['value'], d['unit'], d['roofline']['kernel'][:40], d['roofline']['frac'])"
