#!/bin/bash
# bf16 fused backward occupancy variants: 2-slot weight-gradient ring
# (POSE6D_WGRAD_STAGES=2) and / or a 3-slot data-gradient ring for 4-slot plans
# (POSE6D_BWD_BF16_DS4=3).  Conv tests on the first variant, bf16 step A/B per variant.
TAG=${1:-r05bfr}
VARS=${2:-"ws2 ds3 wd"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
first=${VARS%% *}
POSE6D_LIB=ab/libpose6d_$first.so timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in $VARS; do
  echo "== $v"
  bash tools/ab_lib.sh $OUT/$v ab/libpose6d_$v.so 2 || exit 1
done
