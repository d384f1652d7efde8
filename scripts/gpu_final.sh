# round-end check of the committed build: smoke(), then the driver's default bench line (with cpu_baseline)
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 3
cut -c1-400 $O/bench_default.json
