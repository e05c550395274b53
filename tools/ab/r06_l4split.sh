#!/bin/bash
# bf16 step: fewer weight-gradient splits on the 128x128 (KxK / stride-2) plans -- less slab traffic for the
# carried reduce: layer4 in one split (l4onesplit), target 128 / 64 workgroups (t128, t64), both (t128l4)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in l4onesplit t128 t64 t128l4; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06l4split_$v ab/libpose6d_$v.so 2 || exit 1
done
