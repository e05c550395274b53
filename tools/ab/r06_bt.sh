#!/bin/bash
# bf16 step: workgroup target of the 128x128 (KxK / stride-2) weight-gradient plans: 144 / 192 / 384 vs 256 (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in bt144 bt192 bt384; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06bt_$v ab/libpose6d_$v.so 2 || exit 1
done
