#!/bin/bash
# Round 4: k_ric DMA ring depth A/B (NLOT_RIC_RING 2 / 3 / 4, unicycle_2nd-only builds) on the step_trace workload
OUT=gpurun_out/r04k
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_branches_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
    -k full_solves > $OUT/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/tests.log; tail -2 $OUT/tests.log; grep "^\[parity\]" $OUT/tests.log | cut -c1-250
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in 2 3 4; do
  d=$OUT/ring$R
  NLOT_LIB=libnlot_ring$R.so timeout -k 10 300 python3 scripts/step_trace.py run 32768 2 32768 $d > $d.log 2>&1 || exit $?
  echo "ring $R: $(grep 'traj/s' $d.log)"
done
python3 scripts/cmp_res.py $OUT/ring2/res.npz $OUT/ring3/res.npz
python3 scripts/cmp_res.py $OUT/ring2/res.npz $OUT/ring4/res.npz
