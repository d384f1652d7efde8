# split-bf16 value kernel: microbenchmark vs the f32-MFMA kernel, GPU tests, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mlpv
export TMPDIR=/tmp
NLOT_MLP=f32 timeout -k 10 120 python scripts/mlp_bench.py > gpurun_out/mlpv/micro_f32.log 2>&1 || exit 1
timeout -k 10 120 python scripts/mlp_bench.py > gpurun_out/mlpv/micro_bf16.log 2>&1 || exit 2
grep -h "value\|full" gpurun_out/mlpv/micro_f32.log gpurun_out/mlpv/micro_bf16.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/mlpv/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/mlpv/tests.log; grep -E "passed|failed|FAIL|Error|assert" gpurun_out/mlpv/tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/mlpv/bench.json 2> gpurun_out/mlpv/bench.err
rc=$?; python -c "import json; d=json.loads(open('gpurun_out/mlpv/bench.json').read().strip().splitlines()[-1]); c=d['config']; print(round(d['value']), 'iter_ms', c['solver_step_kernel_ms_per_step'], 'mlp_ms', c['mlp_ms_per_step'], c['status_counts_rank0'])"; exit $rc
