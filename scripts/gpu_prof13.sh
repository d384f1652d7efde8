# kernel-trace profile of one bench solve (B = 65536), current kernels
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof13b
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof13b/bench.log 2>&1
rc=$?; tail -1 gpurun_out/prof13b/bench.log | cut -c1-200; exit $rc
