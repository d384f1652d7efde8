cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -s > gpurun_out/t12.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t12.log; grep -E "agree|passed|failed|k 20" gpurun_out/t12.log | tail -12
[ $rc -eq 0 ] || exit $rc
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 4 > gpurun_out/phase12_b1.log 2>&1
rc=$?; grep -E "QF|solve" gpurun_out/phase12_b1.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b12.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b12.log; tail -2 gpurun_out/b12.log | cut -c1-300
exit $rc
