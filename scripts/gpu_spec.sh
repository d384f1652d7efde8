cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t13.log 2>&1
rc=$?; tail -1 gpurun_out/t13.log; [ $rc -eq 0 ] || exit $rc
for cfg in "2048 1" "2048 2" "8192 1" "512 1"; do
  set -- $cfg
  NLOT_SPEC_THRESHOLD=$1 NLOT_SPEC_BULK=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/spec_$1_$2.log 2>&1 || exit 1
  echo "thr $1 bulk $2: $(python -c "
import json
l=[x for x in open('gpurun_out/spec_$1_$2.log') if x.startswith('{')][-1]; d=json.loads(l); c=d['config']
print(round(d['value'],1), round(d['ms_per_step']), c['lockstep_global_steps'], round(c['solver_step_kernel_ms_per_step']), round(c['mlp_ms_per_step']))")"
done
