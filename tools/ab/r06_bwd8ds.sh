#!/bin/bash
# bf16 step: the 8-wave fused backward's data-gradient ring forced to 2 or 4 slots vs the per-plan choice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in bwd8ds2 bwd8ds4; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06bwd8_$v ab/libpose6d_$v.so 2 || exit 1
done
