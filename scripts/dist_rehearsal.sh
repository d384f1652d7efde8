#!/bin/bash
# bench.py's multi-rank path with the real solver on a 1-GPU box: 2 ranks share cuda:0 over gloo
# (NLOT_DIST_BACKEND=gloo); sharded seeded instances, barriers, max-over-ranks clock, gather to rank 0.
OUT=${OUT:-gpurun_out/r02r}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
NLOT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 1 --batch 8192 --cpu-sample 0 \
    > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || exit $?
tail -c 800 $OUT/bench_n2_gloo.json
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 8192 --cpu-sample 0 > $OUT/bench_n1_8192.json \
    2> $OUT/bench_n1_8192.err || exit $?
tail -c 300 $OUT/bench_n1_8192.json
