# k_ric v2 (3-stage prefetch ring, incremental delta_w): phase timers, GPU tests, A/B vs v10, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ric2
export TMPDIR=/tmp
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 8 > gpurun_out/ric2/b1.log 2>&1 || exit 1
grep -h RICG gpurun_out/ric2/b1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ric2/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/ric2/tests.log; grep -E "passed|failed|FAIL|Error" gpurun_out/ric2/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/ab_solve.py run gpurun_out/ric2/b.npz 4096 > gpurun_out/ric2/ab.log 2>&1 || exit 4
NLOT_LIB=libnlot_v10.so timeout -k 10 200 python scripts/ab_solve.py run gpurun_out/ric2/a.npz 4096 >> gpurun_out/ric2/ab.log 2>&1; python scripts/ab_solve.py cmp gpurun_out/ric2/a.npz gpurun_out/ric2/b.npz >> gpurun_out/ric2/ab.log 2>&1; cat gpurun_out/ric2/ab.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/ric2/bench.json 2> gpurun_out/ric2/bench.err
rc=$?; cut -c1-900 gpurun_out/ric2/bench.json; exit $rc
