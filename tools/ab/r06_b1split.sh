#!/bin/bash
# B = 1 eval forwards (BN + ReLU epilogue): split-K counts per shape, graph-timed
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ENV="conv_splitk=1;conv_splitk=2;conv_splitk=4;conv_splitk=8;conv_splitk=16"
timeout -k 10 300 python tools/conv_bench.py --graph --B 1 --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 --passes fwdnst --env "$ENV" 2>/dev/null || exit 1
