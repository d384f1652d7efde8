# v17 (corner emission fused into k_iter_b / k_accept): GPU tests, MLP microbenchmark, bench of solver build variants, kernel-trace profile of the default build
#   bash scripts/gpu_r14.sh base ring2 ...   (variant v = libnlot_v.so; base = libnlot.so)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r17
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; grep -E "passed|failed|FAIL|Error|assert" $O/tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/mlp_bench.py > $O/micro.log 2>&1 || exit 3
grep -h "value\|full" $O/micro.log
for v in "$@"; do
  lib=libnlot_$v.so; [ "$v" = base ] && lib=libnlot.so
  NLOT_LIB=$lib timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 5
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; r=d['roofline']; print(sys.argv[2], round(d['value']), 'ms', round(d['ms_per_step']), 'iter_ms', round(c['solver_step_kernel_ms_per_step']), 'mlp_ms', round(c['mlp_ms_per_step']), c['status_counts_rank0'], 'steps', c['lockstep_global_steps'], 'frac', round(r['frac'], 3), 'reused', round(r['forward_reused_frac'], 3), flush=True)" $O/bench_$v.json $v
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > $O/prof_bench.log 2>&1 || exit 7
tail -1 $O/prof_bench.log | cut -c1-200
