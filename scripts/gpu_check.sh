#!/bin/bash
# One GPU check of the tree (run through gpurun): the -m gpu suite, the default bench line, and a
# rocprofv3 kernel-trace summary of a short bench.  Every GPU step has its own time limit and the steps
# are chained with &&, so the first failure ends the call.  OUT names the result directory; PYTEST_K is a
# pytest -k expression (quoted as one argument); SKIP_TESTS / SKIP_BENCH skip a stage; STRESS_BENCH=1 adds a
# bench line of the stress workload.
OUT=${OUT:-gpurun_out/check}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  KARGS=()
  [ -n "$PYTEST_K" ] && KARGS=(-k "$PYTEST_K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread "${KARGS[@]}" \
      > "$OUT/gpu_tests.log" 2>&1
  rc=$?
  echo "pytest exit $rc" >> "$OUT/gpu_tests.log"
  tail -3 "$OUT/gpu_tests.log"
  # a GPU fault / abort / time limit ends the call here (exit 1 = failed tests, 5 = none selected: go on)
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
fi
if [ -n "$STRESS_BENCH" ]; then
  timeout -k 10 600 python -u bench.py --workload stress --steps 1 --warmup 1 > "$OUT/bench_stress.json" \
      2> "$OUT/bench_stress.err" || exit $?
  tail -c 1500 "$OUT/bench_stress.json"
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_stress" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload stress --steps 1 --warmup 0 \
      --cpu-sample 0 > "$GRAFT_REPO_ROOT/$OUT/prof_stress_bench.json" 2>&1) || exit $?
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" && \
  tail -c 1500 "$OUT/bench.json" && \
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --cpu-sample 0 \
      > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2>&1) && \
  find "$OUT/prof" -name "*kernel_stats*"
fi
