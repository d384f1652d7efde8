cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in lds global; do
  NLOT_SLOTS=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/slots_$v.log 2>&1 || exit 1
  echo "$v: $(python -c "
import json
l=[x for x in open('gpurun_out/slots_$v.log') if x.startswith('{')][-1]; d=json.loads(l); c=d['config']
print(round(d['value'],1), round(d['ms_per_step']), c['lockstep_global_steps'], round(c['solver_step_kernel_ms_per_step']), round(c['mlp_ms_per_step']), c['riccati_slots'])")"
done
