# phase timers of k_ric (prof build) at B = 1, then a bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/phric
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 3 > gpurun_out/phric/b1.log 2>&1 || exit 1
grep -h RICG gpurun_out/phric/b1.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/phric/bench.json 2> gpurun_out/phric/bench.err
rc=$?; cut -c1-300 gpurun_out/phric/bench.json; python -c "import json; d=json.loads(open('gpurun_out/phric/bench.json').read().strip().splitlines()[-1]); c=d['config']; print('iter_ms', c['solver_step_kernel_ms_per_step'], 'mlp_ms', c['mlp_ms_per_step'], c['status_counts_rank0'])"; exit $rc
