#!/bin/bash
# fp32 LDS-DMA weight-gradient split target (POSE6D_WGRAD_TARGET_F32_FAST) now that the
# fused fp32 backward holds three workgroups per CU: fp32 step A/B per variant
TAG=${1:-r05ft}
VARS=${2:-"ft384 ft768 ft1024"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in $VARS; do
  echo "== $v"
  bash tools/ab_lib.sh $OUT/$v ab/libpose6d_$v.so 2 fp32 || exit 1
done
