#!/bin/bash
# BN finalize, forward and backward, one workgroup per channel (default build) vs the
# backward on one wave per channel (ab/libpose6d_bwdfinwave.so) vs both one-wave
# (ab/libpose6d_finwave512.so = the round-6 start); steps A/B + the BN GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06fin2}
mkdir -p $OUT
echo "== bf16 step: base vs bwd finalize one-wave"; bash tools/ab_lib.sh $OUT/b1 ab/libpose6d_bwdfinwave.so 3 || exit 1
echo "== bf16 step: base vs both one-wave (round-6 start)"; bash tools/ab_lib.sh $OUT/b2 ab/libpose6d_finwave512.so 3 || exit 1
echo "== fp32 step: base vs both one-wave"; bash tools/ab_lib.sh $OUT/f2 ab/libpose6d_finwave512.so 2 fp32 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bn_fusion.py tests/test_config_parity.py tests/test_bn.py 2>&1 | tail -3
