cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export NLOT_LIB=libnlot_prof.so
timeout -k 10 120 python scripts/phase_prof.py 1 4 > gpurun_out/phase_b1.log 2>&1
rc=$?; tail -14 gpurun_out/phase_b1.log; exit $rc
