cd $GRAFT_REPO_ROOT
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_crop.py tests/test_library.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_s2c.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_s2c.json 2> $OUT/bench_s2c.err || exit $?
