# lane-group Riccati (k_ric): GPU parity tests, A/B against the v10 build, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ric1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ric1/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/ric1/tests.log; grep -E "passed|failed|PASS|FAIL|Error" gpurun_out/ric1/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
NLOT_LIB=libnlot_v10.so timeout -k 10 200 python scripts/ab_solve.py run gpurun_out/ric1/a.npz 4096 > gpurun_out/ric1/ab.log 2>&1 || exit 3
timeout -k 10 200 python scripts/ab_solve.py run gpurun_out/ric1/b.npz 4096 >> gpurun_out/ric1/ab.log 2>&1 || exit 4
python scripts/ab_solve.py cmp gpurun_out/ric1/a.npz gpurun_out/ric1/b.npz >> gpurun_out/ric1/ab.log 2>&1; cat gpurun_out/ric1/ab.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/ric1/bench.json 2> gpurun_out/ric1/bench.err
rc=$?; cut -c1-1500 gpurun_out/ric1/bench.json; exit $rc
