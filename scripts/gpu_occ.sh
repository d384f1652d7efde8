# k_iterate occupancy experiment: waves-per-EU 1 (LDS slots) vs 2/3/4 with HBM slots
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/occ
run() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/occ/$name.json 2> gpurun_out/occ/$name.err
  rc=$?
  python -c "import json,sys; d=json.loads(open('gpurun_out/occ/$name.json').read().strip().splitlines()[-1]); c=d['config']; print('$name', round(d['value']), 'iter_ms', round(c['solver_step_kernel_ms_per_step']), 'mlp_ms', round(c['mlp_ms_per_step']), 'step_ms', round(d['ms_per_step']), c['status_counts_rank0'])"
  return $rc
}
run w1_lds && run w1_hbm NLOT_SLOTS=global && run w2_hbm NLOT_LIB=libnlot_w2.so NLOT_SLOTS=global && run w2_lds NLOT_LIB=libnlot_w2.so && run w3_hbm NLOT_LIB=libnlot_w3.so NLOT_SLOTS=global && run w4_hbm NLOT_LIB=libnlot_w4.so NLOT_SLOTS=global
