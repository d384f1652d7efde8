#!/bin/bash
# r02n: GPU suite on the pipelined step loop, then A/B bench lines (1 timed solve each): the default build,
# the unpipelined host loop (NLOT_PIPE=1), and k_ric ring/occupancy variants; a kernel trace of the default.
OUT=gpurun_out/r02n
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/gpu_tests.log; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python -u bench.py --steps 1 --warmup 1 --cpu-sample 0"
timeout -k 10 300 $B > $OUT/base.json 2> $OUT/base.err || exit $?
NLOT_PIPE=1 timeout -k 10 300 $B > $OUT/pipe1.json 2> $OUT/pipe1.err || exit $?
for v in r1w3 r1w4 r2w3; do
  NLOT_LIB=libnlot_$v.so timeout -k 10 300 $B > $OUT/$v.json 2> $OUT/$v.err || exit $?
done
for f in base pipe1 r1w3 r1w4 r2w3; do python -c "import json,sys; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],1), d['config']['status_counts_rank0'], d['config']['lockstep_global_steps'], round(d['roofline']['avg_launch_ms'],4), round(d['ms_per_step'],1))"; done
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --cpu-sample 0 \
    > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2>&1)
