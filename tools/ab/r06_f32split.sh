#!/bin/bash
# fp32 step: layer4's 3x3 weight gradients (128x128 plans, 144 tiles; default 8 splits = 75 MB of slabs the next launch
# reads back) in one split (f32l4one) or without the doubled target (f32nodouble: 4 splits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in f32l4one f32nodouble; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06f32split_$v ab/libpose6d_$v.so 2 fp32 || exit 1
done
