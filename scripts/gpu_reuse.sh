# forward reuse of the accepted trial point in the full MLP launch: tests, bench with / without reuse
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reuse
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/reuse/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/reuse/tests.log; grep -E "passed|failed|FAIL|Error|assert" gpurun_out/reuse/tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  NLOT_MLP_REUSE=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/reuse/bench_$v.json 2> gpurun_out/reuse/bench_$v.err || exit 5
  python -c "import json; d=json.loads(open('gpurun_out/reuse/bench_$v.json').read().strip().splitlines()[-1]); c=d['config']; r=d['roofline']; print('reuse=$v', round(d['value']), 'iter_ms', round(c['solver_step_kernel_ms_per_step']), 'mlp_ms', round(c['mlp_ms_per_step']), c['status_counts_rank0'], 'steps', c['lockstep_global_steps'], 'full_ms', round(r['avg_launch_ms']*r['launches']))"
done
