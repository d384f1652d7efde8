#!/bin/bash
# Pinned-iterate probe of b6 instance 3 (split-bf16 and fp32 SDF net) and the b2 analytic batch test at tol 1e-4.
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/pin_probe.py --case b6 --inst 3 --kmax 22 > $OUT/probe_bf16.log 2>&1 || exit $?
NLOT_MLP=f32 timeout -k 10 300 python3 -u scripts/pin_probe.py --case b6 --inst 3 --kmax 22 > $OUT/probe_f32.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_solver_gpu.py -k "b2_analytic" > $OUT/b2.log 2>&1
echo "exit $?"
tail -5 $OUT/probe_bf16.log $OUT/probe_f32.log $OUT/b2.log
