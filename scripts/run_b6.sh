#!/bin/bash
# b6 (BASELINE configs[3]) on the GPU: its tests, then one bench line and a kernel-trace profile.
set -o pipefail
OUT=gpurun_out/${OUT_TAG:-r02k}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_b6_gpu.py tests/test_cli_gpu.py -v -s --timeout 300 --timeout-method thread > $OUT/b6_tests.log 2>&1
echo "b6 tests exit $?"; grep -E "PASSED|FAILED|b6 " $OUT/b6_tests.log | head -20
timeout -k 10 600 python -u bench.py --workload b6 --steps 1 --warmup 1 > $OUT/bench_b6.json 2> $OUT/bench_b6.err || exit $?
tail -c 600 $OUT/bench_b6.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_b6" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload b6 --steps 1 --warmup 0 --cpu-sample 0 > "$GRAFT_REPO_ROOT/$OUT/prof_b6_bench.json" 2>&1
