#!/bin/bash
# bf16 step: 3-slot ring for the 128x128 weight gradient (and its 8-wave fused launch) vs 2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_lib.sh gpurun_out/r06ws3 ab/libpose6d_ws3.so 3 || exit 1
