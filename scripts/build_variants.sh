#!/bin/bash
# Experiment builds (never the product): libnlot_<name>.so next to libnlot.so, every source compiled with
# extra -D flags, for A/B runs on the GPU box (NLOT_LIB=libnlot_<name>.so).
#   bash scripts/build_variants.sh ring2 "-DNLOT_RIC_RING=2" inord "-DNLOT_RIC_INORDER"
cd "$(dirname "$0")/../nlotrajectories_amd/csrc" || exit 1
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function -Wno-unused-variable"
pids=()
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  (
    d=build/var/$name; mkdir -p $d
    for f in nlot_capi nlot_mlp nlot_solver; do
      /opt/rocm/bin/hipcc $FLAGS $defs -c -o $d/$f.o $f.hip 2> $d/$f.log || exit 1
    done
    /opt/rocm/bin/hipcc $FLAGS -shared -o ../libnlot_$name.so $d/nlot_capi.o $d/nlot_mlp.o $d/nlot_solver.o || exit 1
    echo "built libnlot_$name.so"
  ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
