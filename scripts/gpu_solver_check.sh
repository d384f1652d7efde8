cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_mlp_gpu.py tests/test_solver_gpu.py -x -q -s > gpurun_out/t2.log 2>&1
echo "pytest exit $?" >> gpurun_out/t2.log
tail -40 gpurun_out/t2.log
