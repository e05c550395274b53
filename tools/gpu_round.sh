#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel summary.
# usage: tools/gpu_round.sh TAG [pytest-args...]
TAG=${1:-r}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf "$@" > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests_$TAG.log
if [ $rc -gt 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1
echo "prof rc=$?" >> $OUT/prof_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/roof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-side --no-fp32 --no-cpu-baseline > $OUT/roof_$TAG.log 2>&1
echo "roof rc=$?" >> $OUT/roof_$TAG.log
