#!/bin/bash
# Round 5: rocprofv3 --kernel-trace --stats over the driver's bench command in the default (constraint-row) form, then
# the HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) over a short solve at bench size, k_ric, the MLP
# launches and the phase kernels (scripts/pmc_traffic.sh).
OUT=gpurun_out/r05c
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 \
    > "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.json" 2> "$GRAFT_REPO_ROOT/$OUT/bench_rocprof.err")
rc=$?
find $OUT/prof -name "*kernel_trace.csv" -delete
echo "rocprof exit $rc"
tail -c 300 $OUT/bench_rocprof.json
[ $rc -ne 0 ] && exit $rc
OUT_TAG=r05c/pmc bash scripts/pmc_traffic.sh || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r05c/pmc gpurun_out/r05c/pmc_traffic_r05_B65536.json | tail -40
