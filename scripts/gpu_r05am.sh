#!/bin/bash
# Stress workload, variable-bound form: the round-4 tree (worktree _r04, its own library and bench.py) against this
# tree, same box
OUT=gpurun_out/r05am
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
(cd _r04 && timeout -k 10 400 python -u bench.py --gpus 1 --workload stress --steps 2 --warmup 1 --cpu-sample 0) > $OUT/stress_r04.json 2> $OUT/stress_r04.err || exit $?
python -c "import json; d=json.load(open('$OUT/stress_r04.json')); print('r04', d['value'], d['config']['status_counts_rank0'], d['config']['solver_step_kernel_ms_per_step'], d['config']['mlp_ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 400 python -u bench.py --gpus 1 --workload stress --bounds variable --steps 2 --warmup 1 --cpu-sample 0 > $OUT/stress_now.json 2> $OUT/stress_now.err || exit $?
python -c "import json; d=json.load(open('$OUT/stress_now.json')); print('now', d['value'], d['config']['status_counts_rank0'], d['config']['solver_step_kernel_ms_per_step'], d['config']['mlp_ms_per_step'], d['roofline']['avg_launch_ms'])"
