cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t4.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t4.log; tail -3 gpurun_out/t4.log
[ $rc -eq 0 ] || exit $rc
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 4 > gpurun_out/phase4_b1.log 2>&1
rc=$?; tail -9 gpurun_out/phase4_b1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 4096 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b4_lds.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b4_lds.log; tail -2 gpurun_out/b4_lds.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
NLOT_SLOTS=global timeout -k 10 300 python bench.py --batch 4096 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b4_hbm.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b4_hbm.log; tail -2 gpurun_out/b4_hbm.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b4_16k.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b4_16k.log; tail -2 gpurun_out/b4_16k.log | cut -c1-200
exit $rc
