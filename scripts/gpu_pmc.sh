# HBM traffic of the MLP kernels from PMC counters: separate FETCH_SIZE and WRITE_SIZE passes (TCC slots),
# kernel-trace only (no runtime/sys trace with --pmc), on the fixed-size microbenchmark
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc/fetch -o run --output-format csv -- python3 scripts/mlp_bench.py > gpurun_out/pmc/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc/write -o run --output-format csv -- python3 scripts/mlp_bench.py > gpurun_out/pmc/write.log 2>&1
rc=$?; find gpurun_out/pmc -name "*.csv" | head; exit $rc
