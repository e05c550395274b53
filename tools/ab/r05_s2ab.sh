#!/bin/bash
# stride-2 data-gradient class order variants (POSE6D_S2_ORDER, POSE6D_S2_EMPTY_EXIT):
# graph-timed dgrad / in-place dgrad / fused backward of the stride-2 convs per build
TAG=${1:-r05s2ab}
VARS=${2:-"s2o s2x"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for dt in f32 bf16; do
  for v in base $VARS; do
    L=""; [ $v != base ] && L="--lib ab/libpose6d_$v.so"
    timeout -k 10 300 python -u tools/conv_bench.py $L --dtype $dt --graph --only 8,14,20,6,12,18 --passes dgrad,dgradip,bwd,bwdip --impls fast --tiles auto > $OUT/${dt}_$v.txt 2>&1 || { tail $OUT/${dt}_$v.txt; exit 1; }
    echo "== $dt $v"; grep -v amdgpu.ids $OUT/${dt}_$v.txt | cut -c1-170
  done
done
