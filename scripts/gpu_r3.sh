# wave solver v3 (LDS Riccati slots): parity tests, then LDS vs HBM slots bench, then a kernel-trace profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t3.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t3.log; tail -3 gpurun_out/t3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 4096 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b3_lds.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b3_lds.log; tail -2 gpurun_out/b3_lds.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
NLOT_SLOTS=global timeout -k 10 300 python bench.py --batch 4096 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b3_hbm.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b3_hbm.log; tail -2 gpurun_out/b3_hbm.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof3_bench.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/prof3_bench.log; tail -2 gpurun_out/prof3_bench.log | cut -c1-300
exit $rc
