#!/bin/bash
# layer3 / layer4 3x3 eval forwards (BN + ReLU epilogue): split-K / tile / ring overrides, graph-timed
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ENV="conv_splitk=2;conv_splitk=4;conv_splitk=8;conv_tile=4;conv_tile=4,conv_splitk=2;conv_tile=4,conv_splitk=4;conv_tile=5,conv_splitk=2;conv_tile=5,conv_splitk=4;conv_tile=0,conv_splitk=4"
timeout -k 10 300 python tools/conv_bench.py --graph --only 16,22,10,18 --passes fwdnst --env "$ENV" 2>/dev/null || exit 1
