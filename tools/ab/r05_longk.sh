#!/bin/bash
# fp32 long-K 1x1 forwards on 2 ring slots vs 3 (variant lk3 = POSE6D_F32_LONGK_2SLOT=0): fp32 step A/B
TAG=${1:-r05lk}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/ab_lib.sh $OUT/f32 ab/libpose6d_lk3.so 3 fp32 || exit 1
