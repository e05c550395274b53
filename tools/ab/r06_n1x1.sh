#!/bin/bash
# bf16 step: layer1's 256 -> 64 1x1 weight gradients (the residual-junction backward launches) at a 128-workgroup
# split target (32 splits, POSE6D_WGRAD_NARROW1X1_TARGET=128) vs the 1x1 default (64 splits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_lib.sh gpurun_out/r06n1x1 ab/libpose6d_n1x1.so 4 || exit 1
