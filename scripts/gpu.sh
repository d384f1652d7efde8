#!/bin/bash
# One parameterised GPU-box runner (replaces the per-call scripts of rounds 2-5, kept in git history).
#
#   gpurun -- bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Each STEP runs under its own time limit; the first failing step ends the call (no retries).  Output goes to
# gpurun_out/TAG/.  Steps:
#   env=VAR=VALUE    export VAR=VALUE for the following steps (unenv=VAR unsets it)
#   suite            python -m pytest tests -m gpu (verbose, per-test timeout)
#   smoke            __graft_entry__.smoke()
#   test=EXPR        python -m pytest tests -m gpu -k EXPR (quote EXPR; spaces as '+')
#   bench=K,W[,ARGS] python bench.py --gpus 1 --steps K --warmup W [ARGS: ','-separated extra arguments]
#   rocprof=K,W      rocprofv3 --kernel-trace --stats over bench.py --steps K --warmup W
#   pmc=K,W,COUNTERS rocprofv3 --pmc COUNTERS (one pass) over bench.py --steps K --warmup W --cpu-sample 0
#   py=SCRIPT[,ARGS] python3 SCRIPT [ARGS]  (a script under scripts/, 600 s limit)
#   sh=SCRIPT[,ARGS] bash SCRIPT [ARGS]     (900 s limit)
#   rehearse=K,W[,B] NLOT_DIST_BACKEND=gloo bench.py --gpus 2 (self-launched ranks sharing this GPU), B per rank
#   regress          the restoration grid-bound test against libnlot_regress.so (scripts/resto_bound_regress.sh): must fail
TAG=$1
shift
OUT=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  IFS=, read -r -a A <<< "$arg"
  log=$OUT/$n.$name.log
  echo "[gpu.sh] step $n: $step" >&2
  case $name in
    env)  # env=VAR=VALUE: exported for the following steps
      export "$arg"; rc=0 ;;
    unenv)
      unset "$arg"; rc=0 ;;
    suite)
      timeout -k 10 1150 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > "$log" 2>&1
      rc=$?; tail -1 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; tail -1 "$log" | cut -c1-200 ;;
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
        -k "${arg//+/ }" > "$log" 2>&1
      rc=$?; tail -1 "$log" ;;
    bench)
      extra=("${A[@]:2}")
      timeout -k 10 900 python -u bench.py --gpus 1 --steps "${A[0]}" --warmup "${A[1]}" "${extra[@]}" \
        > "$OUT/$n.bench.json" 2> "$log"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], d['config']['status_counts_rank0'], 'frac', r['frac'], r['avg_launch_ms'])" "$OUT/$n.bench.json" ;;
    rehearse)  # bench.py --gpus 2 with no launcher: it starts 2 ranks itself; gloo collectives, both ranks on this GPU
      NLOT_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps "${A[0]}" --warmup "${A[1]}" \
        --batch "${A[2]:-4096}" --slots "${A[2]:-4096}" > "$OUT/$n.bench.json" 2> "$log"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rehearsal n_gpus', d['n_gpus'], d['config']['process_group'], d['value'], [r['status_counts'] for r in d['config']['per_rank']])" "$OUT/$n.bench.json" ;;
    rocprof)
      # the kernel trace is too large to copy back: it stays in /tmp, the --stats summary comes back
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/rocprof_$TAG" -o run -- \
        python3 bench.py --gpus 1 --steps "${A[0]}" --warmup "${A[1]}" --cpu-sample 0 > "$OUT/$n.bench.json" 2> "$log"
      rc=$?
      find "/tmp/rocprof_$TAG" -name "*kernel_stats.csv" -exec cp {} "$OUT/$n.kernel_stats.csv" \; ;;
    pmc)
      timeout -s KILL 600 rocprofv3 --pmc "${A[@]:2}" -d "/tmp/pmc_${TAG}_$n" -o run -- \
        python3 bench.py --gpus 1 --steps "${A[0]}" --warmup "${A[1]}" --cpu-sample 0 > "$OUT/$n.bench.json" 2> "$log"
      rc=$? ;;
    regress)  # scripts/resto_bound_regress.sh's library: the restoration grid-bound test must FAIL on it
      NLOT_LIB=libnlot_regress.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 500 \
        --timeout-method thread -k resto_grid_bound > "$log" 2>&1
      r=$?; tail -1 "$log"
      if [ $r -eq 1 ]; then echo "[gpu.sh] regress: the test failed on the old clamp, as it must"; rc=0; else rc=1; fi ;;
    sh)
      timeout -k 10 900 bash "${A[@]}" > "$log" 2>&1
      rc=$?; tail -3 "$log" ;;
    py)
      timeout -k 10 600 python3 -u "${A[@]}" > "$log" 2>&1
      rc=$?; tail -3 "$log" ;;
    *)
      echo "[gpu.sh] unknown step $step" >&2; exit 2 ;;
  esac
  echo "[gpu.sh] step $n ($name) exit $rc" >&2
  [ $rc -ne 0 ] && exit $rc
done
exit 0
