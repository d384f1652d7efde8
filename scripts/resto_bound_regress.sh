#!/bin/bash
# Demonstrates that tests/test_resto_gpu.py::test_resto_grid_bound_same_results catches the round-5 restoration-list
# bug: builds libnlot_regress.so (benchmark 6's dynamics only, NLOT_ONLY_DYN=5) from a copy of nlot_solver.hip with
# k_ric<DYN, true>'s list count clamped to its grid bound again (the line before 4e8db73).  Run here (CPU, build) and
# then on the GPU box:  NLOT_LIB=libnlot_regress.so python -m pytest tests -m gpu -k resto_grid_bound  -> must FAIL.
# Never the product; delete the library afterwards.
set -e
cd "$(dirname "$0")/../nlotrajectories_amd/csrc"
mkdir -p build/regress
sed 's/const int nlist = RESTO ? \*nact : std::min(n_active, \*nact);/const int nlist = std::min(n_active, *nact);  \/\/ REGRESSION: 4e8db73^/' \
    nlot_solver.hip > build/regress/nlot_solver.hip
grep -q "REGRESSION: 4e8db73" build/regress/nlot_solver.hip
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-function"
/opt/rocm/bin/hipcc $HIPFLAGS -DNLOT_ONLY_DYN=5 -I. -c -o build/regress/nlot_solver.o build/regress/nlot_solver.hip
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o ../libnlot_regress.so build/nlot_capi.o build/nlot_mlp.o build/regress/nlot_solver.o build/nlot_rrt.o
echo built ../libnlot_regress.so
