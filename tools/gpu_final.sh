#!/bin/bash
# Round-end measurement: GPU tests + bench + rocprof stats (tools/gpu_round.sh), PMC
# traffic / MFMA-busy passes (tools/pmc_round.sh), then one-box A/B of the eval fusions.
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh $TAG || exit $?
bash tools/pmc_round.sh $TAG || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab_env.py POSE6D_EVAL_DUAL=0 POSE6D_EVAL_DUAL=1 3 > gpurun_out/ab_dual.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ab_env.py POSE6D_HEAD_BN_FUSE=0 POSE6D_HEAD_BN_FUSE=1 3 > gpurun_out/ab_head.txt 2>&1
