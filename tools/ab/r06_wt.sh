#!/bin/bash
# bf16 step: workgroup targets of the 64x64 weight-gradient plans: 1x1 (POSE6D_WGRAD_TARGET 128 / 192 vs 256) and
# KxK (POSE6D_WGRAD_TARGET_KXK 192 vs 256: layer1's 3x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in wt128 wt192 wk192; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06wt_$v ab/libpose6d_$v.so 2 || exit 1
done
