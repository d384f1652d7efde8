cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_solver_gpu.py -x -q > gpurun_out/t_wave2.log 2>&1
echo "tests exit $?" >> gpurun_out/t_wave2.log
tail -2 gpurun_out/t_wave2.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --batch 4096 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof2_bench.log 2>&1
echo "exit $?" >> gpurun_out/prof2_bench.log
tail -2 gpurun_out/prof2_bench.log | cut -c1-400
