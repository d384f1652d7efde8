cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof6
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof6_bench.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/prof6_bench.log; tail -2 gpurun_out/prof6_bench.log | cut -c1-200
exit $rc
