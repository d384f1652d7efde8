#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs: 3 + 2 TCC counters) over a short metric solve
# at bench size (scripts/pmc_solve.py: B = 65536, 8 iterations), the solver's and MLP kernels; summarised per unit
# (solve, point, instance-iteration) by scripts/pmc_traffic.py on the box.  The per-dispatch counter CSVs stay in
# /tmp (too large to copy back); gpurun_out/TAG/ gets the summary and the runs' solver statistics.
#     bash scripts/pmc_traffic.sh TAG
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${1:-r06pmc}
OUT="$R/gpurun_out/$TAG"
WORK=/tmp/pmc_$TAG
mkdir -p "$OUT" "$WORK"
export TMPDIR=/tmp
cd /tmp || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_ric|mlp_bf16|k_iter_a|k_iter_b|k_accept|k_resto" \
      -d "$WORK/pmc_$C" -o run \
      --output-format csv -- python3 "$R/scripts/pmc_solve.py" ${PMC_BATCH:-65536} ${PMC_ITERS:-8} \
      > "$WORK/pmc_${C}_stats.json" 2> "$WORK/pmc_${C}.err" || exit $?
  cp "$WORK/pmc_${C}_stats.json" "$OUT/"
  echo "pass $C done"
done
python3 "$R/scripts/pmc_traffic.py" "$WORK" "$OUT/pmc_traffic_B65536.json" > /dev/null || exit $?
echo "summary: $OUT/pmc_traffic_B65536.json"
