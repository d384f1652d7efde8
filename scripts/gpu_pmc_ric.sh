# SQ counters of the solver kernels (k_ric, k_iter_a, ...): two separate passes, kernel-trace only;
# the raw per-dispatch CSVs are aggregated per kernel on the box (scripts/pmc_agg.py) and dropped
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcr
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d /tmp/pmcr/p1 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/pmcr/p1.log 2>&1 || exit 2
python scripts/pmc_agg.py $(find /tmp/pmcr/p1 -name "*counter_collection.csv") gpurun_out/pmcr/p1.json || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --kernel-trace -d /tmp/pmcr/p2 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/pmcr/p2.log 2>&1 || exit 3
python scripts/pmc_agg.py $(find /tmp/pmcr/p2 -name "*counter_collection.csv") gpurun_out/pmcr/p2.json || exit 5
rm -rf /tmp/pmcr
