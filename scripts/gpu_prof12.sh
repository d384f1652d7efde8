cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof12
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof12_bench.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/prof12_bench.log; tail -2 gpurun_out/prof12_bench.log | cut -c1-200; exit $rc
