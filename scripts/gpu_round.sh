# one GPU session: tests, a short bench, and a kernel-trace profile of the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > gpurun_out/tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/tests.log
tail -5 gpurun_out/tests.log
timeout -k 10 600 python bench.py --batch ${BENCH_B:-4096} --steps 1 --warmup 1 --cpu-sample 16 > gpurun_out/bench.log 2>&1
echo "bench exit $?" >> gpurun_out/bench.log
tail -3 gpurun_out/bench.log
