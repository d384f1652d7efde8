OUT=gpurun_out/r03n; mkdir -p $OUT
NLOT_LIB=libnlot_tune.so timeout -k 10 120 python -u scripts/pmc_solve.py 16 4 > $OUT/prof_B16.log 2>&1 || exit 1
NLOT_LIB=libnlot_tune.so timeout -k 10 200 python -u scripts/pmc_solve.py 65536 3 > $OUT/prof_B65536.log 2>&1 || exit 1
grep -c RICG $OUT/prof_B16.log $OUT/prof_B65536.log
