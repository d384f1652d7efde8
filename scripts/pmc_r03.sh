#!/bin/bash
# PMC passes (one counter group per run, MI355X_MICROARCH.md: FETCH_SIZE 3 TCC counters, WRITE_SIZE 2) over a
# short metric solve at bench size (B = 65536, 8 iterations): HBM bytes per point of the MLP launches and per
# Newton solve of k_ric.  Kernel trace + stats in a separate run.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${OUT_TAG:-r03pmc}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B=${PMC_BATCH:-65536}
IT=${PMC_ITERS:-8}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/scripts/pmc_solve.py" $B $IT > "$OUT/trace_stats.json" 2> "$OUT/trace.err" || exit $?
echo "trace done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_ric|mlp_bf16" -d "$OUT/pmc_$C" -o run \
      --output-format csv -- python3 "$R/scripts/pmc_solve.py" $B $IT > "$OUT/pmc_${C}_stats.json" \
      2> "$OUT/pmc_${C}.err" || exit $?
  echo "pass $C done"
done
