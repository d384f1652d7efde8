cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in NO_SINCOS NO_REV; do
  echo "== $V"; NLOT_LIB=libnlot_exp_$V.so timeout -k 10 120 python scripts/mlp_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
