#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab_env.py POSE6D_EVAL_DUAL=0 POSE6D_EVAL_DUAL=1 4 > gpurun_out/ab_dual.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab_env.py POSE6D_HEAD_BN_FUSE=0 POSE6D_HEAD_BN_FUSE=1 4 > gpurun_out/ab_head.txt 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --graph --passes fwdact,fwdactres --impls fast --tiles auto --stages auto,2,3,4 \
  --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 > gpurun_out/act_stages.txt 2>&1
