#!/bin/bash
# Upper bound of the value-MLP epilogue's cost: the standalone launches (scripts/mlp_bench.py, 3.3 M points) with the
# epilogue's per-row bias / output-weight LDS reads replaced by constants (libnlot_mlpexp.so, wrong values) against
# the product library
OUT=gpurun_out/r05ac
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
for v in libnlot.so libnlot_mlpexp.so libnlot.so libnlot_mlpexp.so; do
  NLOT_LIB=$v timeout -k 10 120 python3 scripts/mlp_bench.py > $OUT/$v.log 2>&1 || exit $?
  echo "$v: $(tr '\n' ' ' < $OUT/$v.log)"
done
