#!/bin/bash
# fp32 fused backward at three workgroups per CU: smaller weight-gradient stages
# (POSE6D_BWD_F32_MS) and data-gradient ring (POSE6D_BWD_F32_DS4) variants.
# Conv tests on the first variant, fp32 step A/B (tools/fp32_step.py) for each.
TAG=${1:-r05f32r}
VARS=${2:-"f32a f32b f32c"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
first=${VARS%% *}
POSE6D_LIB=ab/libpose6d_$first.so timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in $VARS; do
  echo "== $v"
  bash tools/ab_lib.sh $OUT/$v ab/libpose6d_$v.so 2 fp32 || exit 1
done
