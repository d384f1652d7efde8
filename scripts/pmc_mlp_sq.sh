#!/bin/bash
# SQ PMC passes (8 SQ counters + GRBM each, separate runs, --kernel-trace style collection only) over the MLP
# microbenchmark (scripts/mlp_bench.py: full and value launches on 3.3 M points): where a wave's cycles go and the
# instruction mix of mlp_bf16<128,*>.  Also lists the available counters once (rocprofv3 -L).
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${OUT_TAG:-r04mlp}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "list failed"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "mlp_bf16" -d "$OUT/pmc$i" -o run --output-format csv \
      -- python3 "$R/scripts/mlp_bench.py" > "$OUT/pmc$i.log" 2>&1 || exit $?
  echo "pass $i done"
  i=$((i + 1))
done
