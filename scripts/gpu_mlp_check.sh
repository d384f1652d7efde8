cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m3 -E "Name:.*gfx|Marketing" > gpurun_out/rocminfo.txt 2>&1 || true
nproc > gpurun_out/nproc.txt
timeout -k 10 300 python -m pytest tests/test_mlp_gpu.py -x -q > gpurun_out/t1.log 2>&1
echo "pytest exit $?" >> gpurun_out/t1.log
tail -30 gpurun_out/t1.log
