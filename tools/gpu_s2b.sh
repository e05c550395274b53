cd $GRAFT_REPO_ROOT
OUT=gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_s2b.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench_s2b.json 2> $OUT/bench_s2b.err || exit $?
bash tools/pmc_round.sh s2b
