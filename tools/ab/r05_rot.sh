#!/bin/bash
# Stride-2 data gradient with the parity-class order rotated per tile (POSE6D_S2_ROTATE):
# conv tests + config parity on the variant, graph-timed stride-2 convs per build,
# bf16 and fp32 step A/B.
TAG=${1:-r05rot}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
POSE6D_LIB=ab/libpose6d_rot.so timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for dt in f32 bf16; do
  for v in base rot; do
    L=""; [ $v != base ] && L="--lib ab/libpose6d_$v.so"
    timeout -k 10 300 python -u tools/conv_bench.py $L --dtype $dt --graph --only 8,14,20,6,12,18 --passes dgrad,dgradip,bwd,bwdip --impls fast --tiles auto > $OUT/${dt}_$v.txt 2>&1 || { tail $OUT/${dt}_$v.txt; exit 1; }
    echo "== $dt $v"; grep -v amdgpu.ids $OUT/${dt}_$v.txt | cut -c1-170
  done
done
bash tools/ab_lib.sh $OUT/bf16 ab/libpose6d_rot.so 2 || exit 1
bash tools/ab_lib.sh $OUT/f32 ab/libpose6d_rot.so 2 fp32 || exit 1
