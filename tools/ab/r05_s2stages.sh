#!/bin/bash
# stride-2 3x3 data-gradient ring depths after the class rotation (tuned stages, no rebuild)
TAG=${1:-r05s2st}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for dt in f32 bf16; do
  timeout -k 10 300 python -u tools/conv_bench.py --dtype $dt --graph --only 6,12,18 --passes dgrad --impls fast --tiles auto,0,3,4 --stages auto,2,3,4 > $OUT/$dt.txt 2>&1 || { tail $OUT/$dt.txt; exit 1; }
  echo "== $dt"; grep -v amdgpu.ids $OUT/$dt.txt | cut -c1-400
done
