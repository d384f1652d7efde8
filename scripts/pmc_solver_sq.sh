#!/bin/bash
# SQ PMC passes (8 SQ + 1 GRBM counters each, separate runs) over a short metric solve at bench size
# (scripts/pmc_solve.py: B = 65536, 8 iterations): where the waves of the phase-machine kernels (k_iter_a,
# k_iter_b, k_accept) and of k_ric spend their cycles, and their instruction mix.  Summarised by
# scripts/pmc_sq_summary.py.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${OUT_TAG:-r04sq}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
RX="k_iter_a|k_iter_b|k_accept|k_ric|mlp_bf16"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P2="SQ_INSTS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" -d "$OUT/pmc$i" -o run --output-format csv \
      -- python3 "$R/scripts/pmc_solve.py" ${PMC_BATCH:-65536} ${PMC_ITERS:-8} > "$OUT/pmc$i.log" 2>&1 || exit $?
  echo "pass $i done"
  i=$((i + 1))
done
