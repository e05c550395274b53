#!/bin/bash
OUT=$GRAFT_REPO_ROOT/gpurun_out/kg_$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/kg_check.py f32 > $OUT/check_f32.txt 2>&1 || exit $?
timeout -k 10 300 python tools/kg_check.py bf16 > $OUT/check_bf16.txt 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --graph --dtype f32 --passes fwd,fwdact --impls fast --tiles auto,6 \
  --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 > $OUT/f32.txt 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --graph --dtype bf16 --passes fwd,fwdact --impls fast --tiles auto,6 \
  --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 > $OUT/bf16.txt 2>&1
