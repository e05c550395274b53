#!/bin/bash
# One build -> measure iteration on the GPU box: GPU tests, conv epilogue sweep, bench.
# usage: tools/gpu_iter.sh TAG [conv_bench passes]
TAG=${1:-i}
PASSES=${2:-fwdns,fwdact,fwdactres}
OUT=$GRAFT_REPO_ROOT/gpurun_out/iter_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/conv_bench.py --graph --passes $PASSES --impls fast --tiles auto \
  --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 > $OUT/conv.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
