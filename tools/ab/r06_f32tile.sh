#!/bin/bash
# fp32 step: wider 128x128 (8-wave) tile rules for the fp32 forwards / data gradients (POSE6D_F32_TILE_RULE 1, 2) vs the
# round-2 rule (K >= 512, 192 <= 128x128 workgroups < 384)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in f32t1 f32t2; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06f32tile_$v ab/libpose6d_$v.so 2 fp32 || exit 1
done
