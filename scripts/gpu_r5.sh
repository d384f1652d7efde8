cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -x -q -s > gpurun_out/t5.log 2>&1
rc=$?; echo "tests exit $rc" >> gpurun_out/t5.log; grep -E "agree|passed|failed|Error" gpurun_out/t5.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/b5_adap.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b5_adap.log; tail -2 gpurun_out/b5_adap.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 1 --cpu-sample 0 --mu-strategy monotone > gpurun_out/b5_mono.log 2>&1
rc=$?; echo "exit $rc" >> gpurun_out/b5_mono.log; tail -2 gpurun_out/b5_mono.log | cut -c1-200
exit $rc
