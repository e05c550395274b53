#!/bin/bash
# layer1 256->64 / 256->128 1x1 fused backward with the junction gradient (dres), isolated:
# split / order / separate-launch overrides, warm and behind a 512 MB write
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ENV="wgrad_splits=16;wgrad_splits=32;wgrad_splits=128;wgrad_splits=256;bwd_order=0;bwd_separate=1;wgrad_stages=2;wgrad_stages=4"
timeout -k 10 300 python tools/conv_bench.py --graph --only 4,5,3,9 --passes bwd,bwdres --env "$ENV" 2>/dev/null || exit 1
timeout -k 10 300 python tools/conv_bench.py --graph --only 4,5 --passes bwdrescold --env "$ENV" 2>/dev/null || exit 1
