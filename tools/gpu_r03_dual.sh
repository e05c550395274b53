#!/bin/bash
# BN-reduce epilogue + dual BN backward: tests, interleaved step A/B, then the profiling run
set -o pipefail
TAG=${1:-r03q}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_fusion.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.bwd_conv_bn_reduce > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
[ "${2:-}" = "prof" ] && bash tools/gpu_r03_prof.sh ${TAG}p
echo done
