#!/bin/bash
# One SQ PMC pass (7 counters) over k_ric in a short metric solve (B = 16384): where a k_ric wave's cycles go
# (issuing / waiting on memory or barriers / issue-stalled) and its instruction mix.  Summarised by
# scripts/pmc_kric_sq.py into profiles/r02/kric_sq.json.
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/${OUT_TAG:-r02q}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
    --kernel-include-regex "k_ric" -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 \
    --cpu-sample 0 --batch 16384 > "$OUT/pmc_sq_bench.json" 2> "$OUT/pmc_sq_bench.err" || exit $?
echo "pass SQ done"
