cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --batch 131072 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b64k.log 2>&1
rc=$?; tail -1 gpurun_out/b64k.log | cut -c1-150; exit $rc
