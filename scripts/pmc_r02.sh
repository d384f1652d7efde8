#!/bin/bash
# PMC passes (one counter group per run) over a short metric solve: HBM bytes of k_ric and the MLP kernels.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${OUT_TAG:-r02j}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_ric|mlp_bf16|mlp_stream" -d "$OUT/pmc_$C" -o run \
      --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-sample 0 --batch ${PMC_BATCH:-2048} \
      > "$OUT/pmc_${C}_bench.json" 2> "$OUT/pmc_${C}_bench.err" || exit $?
  echo "pass $C done"
done
