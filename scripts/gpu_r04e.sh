#!/bin/bash
# Round 4: MLP kernel rework (templated input layer, 2 waves/SIMD full launch) — MLP parity tests, microbenchmark
# A/B against the previous kernel (libnlot_base.so), and a solve A/B on the step_trace workload (bitwise compare).
OUT=gpurun_out/r04e
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mlp_gpu.py -m gpu -v -s --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in libnlot_base.so libnlot.so; do
    NLOT_LIB=$lib timeout -k 10 120 python3 scripts/mlp_bench.py > $OUT/mlp_${lib%.so}.log 2>&1 || exit $?
    echo "$lib"; cat $OUT/mlp_${lib%.so}.log
done
for lib in libnlot_base.so libnlot.so; do
    d=$OUT/solve_${lib%.so}
    NLOT_LIB=$lib timeout -k 10 300 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
    echo "$lib: $(grep 'traj/s' $d.log)"
done
python3 scripts/cmp_res.py $OUT/solve_libnlot_base/res.npz $OUT/solve_libnlot/res.npz
