#!/bin/bash
# bf16 step: 128x128 weight-gradient target 192 (3 rounds) and 160 / 224 vs 256 (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== base vs bt192"; bash tools/ab_lib.sh gpurun_out/r06bt2_bt192 ab/libpose6d_bt192.so 3 || exit 1
for v in bt160 bt224; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06bt2_$v ab/libpose6d_$v.so 2 || exit 1
done
