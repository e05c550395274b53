#!/bin/bash
# fp32 forward / data-gradient ring-depth sweep over the ResNet50 conv shapes (bs32,
# graph-timed; tuned stage counts through pose6d_tuning_t, no rebuild)
TAG=${1:-r05f32st}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u tools/conv_bench.py --dtype f32 --graph --passes fwd,dgrad --impls fast --tiles auto --stages auto,2,3,4 > $OUT/sweep.txt 2>&1 || { tail $OUT/sweep.txt; exit 1; }
grep -v amdgpu.ids $OUT/sweep.txt | cut -c1-250
