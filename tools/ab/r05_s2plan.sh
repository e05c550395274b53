#!/bin/bash
# fp32 KxK stride-2 data-gradient plan (64x64, 4 slots) vs the generic rules (variant
# s2old = POSE6D_F32_S2_PLAN=0): fp32 step A/B
TAG=${1:-r05s2p}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/ab_lib.sh $OUT/f32 ab/libpose6d_s2old.so 2 fp32 || exit 1
