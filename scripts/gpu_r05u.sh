#!/bin/bash
# Round 5 (final tree): rocprofv3 --kernel-trace --stats over the driver's bench command in the default (constraint-row) form, then
# the HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) over a short solve at bench size, k_ric, the MLP
# launches and the phase kernels (scripts/pmc_traffic.sh).
OUT=gpurun_out/r05u
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
OUT_TAG=r05u/pmc bash scripts/pmc_traffic.sh || exit $?
python3 scripts/pmc_traffic.py gpurun_out/r05u/pmc gpurun_out/r05u/pmc_traffic_r05u_B65536.json | tail -40
python3 scripts/rocprof_fracs.py $(find gpurun_out/r05u/prof -name "*kernel_stats.csv" | head -1) gpurun_out/r05u/bench_rocprof.json gpurun_out/r05u/mlp_dispatch_fracs_r05u.json | tail -5
