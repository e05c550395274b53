#!/bin/bash
# fp32 128x128 weight gradient at three workgroups per CU: 16-pixel stages
# (POSE6D_WGRAD_F32_MS128=16) + half-tile acc staging.  Conv tests on the variant,
# graph-timed KxK weight gradients (2 / 3 slots), fp32 step A/B.
TAG=${1:-r05ms16}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
POSE6D_LIB=ab/libpose6d_ms16.so timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in base ms16; do
  L=""; [ $v != base ] && L="--lib ab/libpose6d_$v.so"
  timeout -k 10 300 python -u tools/conv_bench.py $L --dtype f32 --graph --only 2,6,10,12,16,18,22 --passes wgrad --tiles auto --wgrad-env "wgrad_stages=3" > $OUT/w_$v.txt 2>&1 || { tail $OUT/w_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/w_$v.txt | cut -c1-120
done
bash tools/ab_lib.sh $OUT/ab ab/libpose6d_ms16.so 2 fp32 || exit 1
