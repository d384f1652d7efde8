#!/bin/bash
# r02w: the stress workload under the default bench settings (K = 4 continuous), and the 2-rank gloo rehearsal of
# the multi-rank path with continuous batching (2 timed batches per rank).
OUT=gpurun_out/r02w
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
NLOT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 2 --warmup 1 --batch 8192 --cpu-sample 0 \
    > $OUT/bench_n2_gloo_cont.json 2> $OUT/bench_n2_gloo_cont.err || exit $?
tail -c 300 $OUT/bench_n2_gloo_cont.json
timeout -k 10 900 python -u bench.py --workload stress > $OUT/stress.json 2> $OUT/stress.err || exit $?
tail -c 300 $OUT/stress.json
timeout -k 10 900 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
tail -c 300 $OUT/bench_default.json
