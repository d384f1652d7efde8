#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs: 3 + 2 TCC counters) over a short metric solve
# at bench size (scripts/pmc_solve.py: B = 65536, 8 iterations), kernels k_ric and mlp_bf16 only; summarised per unit
# (solve, point) by scripts/pmc_traffic.py.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${1:-${OUT_TAG:-r06pmc}}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_ric|mlp_bf16|k_iter_a|k_iter_b|k_accept|k_resto" \
      -d "$OUT/pmc_$C" -o run \
      --output-format csv -- python3 "$R/scripts/pmc_solve.py" ${PMC_BATCH:-65536} ${PMC_ITERS:-8} \
      > "$OUT/pmc_${C}_stats.json" 2> "$OUT/pmc_${C}.err" || exit $?
  echo "pass $C done"
done
