#!/bin/bash
# GPU tests, bench, then a kernel trace of replayed training steps (tools/step_trace.sh).
TAG=${1:-i}
OUT=$GRAFT_REPO_ROOT/gpurun_out/iter_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
bash tools/step_trace.sh $TAG
