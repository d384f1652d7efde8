# phase timers of k_ric (prof build) at B = 1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/phric
NLOT_LIB=libnlot_prof.so timeout -k 10 120 python scripts/phase_prof.py 1 3 > gpurun_out/phric/b1.log 2>&1 || exit 1
grep -h RICG gpurun_out/phric/b1.log
