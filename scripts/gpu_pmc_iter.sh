# k_iterate instruction mix (SQ counters, two separate passes, kernel-trace only) + phase timers at B=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmci
export TMPDIR=/tmp
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 12 > gpurun_out/pmci/phase_b1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/pmci/p1 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/pmci/p1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH --kernel-trace -d gpurun_out/pmci/p2 -o run --output-format csv -- python3 bench.py --batch 16384 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/pmci/p2.log 2>&1 || exit 3
find gpurun_out/pmci -name "*.csv" | head
