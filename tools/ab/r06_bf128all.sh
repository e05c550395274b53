#!/bin/bash
# bf16 step: the 128x128 weight gradient on every eligible conv incl. the stride-1 1x1s (POSE6D_WGRAD_BF128=2), after
# the round-6 split retune, vs KxK / stride-2 only (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_lib.sh gpurun_out/r06bf128all ab/libpose6d_bf128all.so 2 || exit 1
