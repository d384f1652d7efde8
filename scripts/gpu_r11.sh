cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -s > gpurun_out/t11.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t11.log; grep -E "agree|passed|failed|k 20" gpurun_out/t11.log | tail -12
[ $rc -eq 0 ] || exit $rc
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 4 > gpurun_out/phase11_b1.log 2>&1
rc=$?; tail -9 gpurun_out/phase11_b1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b11_adap.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b11_adap.log; tail -2 gpurun_out/b11_adap.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
NLOT_SLOTS=global timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b11_adap_hbm.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b11_adap_hbm.log; tail -2 gpurun_out/b11_adap_hbm.log | cut -c1-200
exit $rc
