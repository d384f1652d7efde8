# k_ric v3 (stage inputs by global->LDS DMA ring): phase timers, GPU tests, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ric3
export TMPDIR=/tmp
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 3 > gpurun_out/ric3/b1.log 2>&1 || exit 1
grep -h RICG gpurun_out/ric3/b1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ric3/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/ric3/tests.log; grep -E "passed|failed|FAIL|Error" gpurun_out/ric3/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/ric3/bench.json 2> gpurun_out/ric3/bench.err
rc=$?; python -c "import json; d=json.loads(open('gpurun_out/ric3/bench.json').read().strip().splitlines()[-1]); c=d['config']; print(round(d['value']), 'iter_ms', c['solver_step_kernel_ms_per_step'], 'mlp_ms', c['mlp_ms_per_step'], c['status_counts_rank0'])"; exit $rc
