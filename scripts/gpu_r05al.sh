#!/bin/bash
# Step timeline after k_step_end (one batch of 32,768, scripts/timeline.py), and the stress workload in the
# variable-bound form (is the round-5 stress status mix the NLP form?)
OUT=gpurun_out/r05al
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o trace -- python3 $GRAFT_REPO_ROOT/scripts/step_trace.py run 32768 1 32768 $GRAFT_REPO_ROOT/$OUT/traced > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $T --out $OUT/timeline.json > /dev/null || exit $?
python3 -c "
import json; d=json.load(open('$OUT/timeline.json'))
print('wall', round(d['wall_us_per_step'],1)); print({k: [round(x,1) for x in v[:2]] for k,v in d['launch_start_end_us_from_step_start'].items() if v[2] > 100}); print(d['waits_us'])"
gzip -c $T > $OUT/kernel_trace.csv.gz
rm -f $T
timeout -k 10 400 python -u bench.py --gpus 1 --workload stress --bounds variable --cpu-sample 0 > $OUT/bench_stress_var.json 2> $OUT/bench_stress_var.err || exit $?
python -c "import json; d=json.load(open('$OUT/bench_stress_var.json')); print('stress variable bounds', d['value'], d['config']['status_counts_rank0'])"
