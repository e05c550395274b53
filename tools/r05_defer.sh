#!/bin/bash
# Deferred batched weight gradients: tests, A/B on the bf16 step, kernel trace with it on
TAG=${1:-r05d2}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_deferred_wgrad.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.defer_wgrad --rounds 9 > $OUT/ab_bf16.txt 2>&1 || { tail $OUT/ab_bf16.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_bf16.txt
