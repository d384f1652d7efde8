set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest tests/test_solver_gpu.py -k tiny -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r02i/tiny.log 2>&1; echo "tiny exit $?"; grep -E "^tiny|PASSED|FAILED" gpurun_out/r02i/tiny.log
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/r02i/base.json 2> gpurun_out/r02i/base.err &&
NLOT_LIB=libnlot_wpe2.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/r02i/wpe2.json 2> gpurun_out/r02i/wpe2.err
