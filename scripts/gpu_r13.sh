# round-1 re-entry check: GPU parity tests, default bench (with CPU baseline), kernel-trace profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof13
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t13.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t13.log; grep -E "passed|failed|PASS|FAIL" gpurun_out/t13.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/b13.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b13.log; tail -2 gpurun_out/b13.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof13_bench.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/prof13_bench.log; tail -2 gpurun_out/prof13_bench.log | cut -c1-200; exit $rc
