#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06k}
mkdir -p $OUT
bash tools/ab/r06_add2.sh ${1:-r06k}_add || exit 1
bash tools/ab_lib.sh $OUT/ab_all128 ab/libpose6d_all128.so 3 || exit 1
bash tools/ab/r06_breakdown.sh ${1:-r06k}_bd ab/libpose6d_all128.so || exit 1
