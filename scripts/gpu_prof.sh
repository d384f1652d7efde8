cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --batch ${BENCH_B:-1024} --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_bench.log 2>&1
echo "exit $?" >> gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
tail -2 gpurun_out/prof_bench.log
