cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_mlp_gpu.py -q > gpurun_out/mlpt.log 2>&1 && \
timeout -k 10 120 python scripts/mlp_bench.py > gpurun_out/mlpb.log 2>&1
rc=$?; tail -2 gpurun_out/mlpt.log; cat gpurun_out/mlpb.log; exit $rc
