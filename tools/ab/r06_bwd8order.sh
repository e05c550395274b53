#!/bin/bash
# bf16 step: the 8-wave fused backward with the weight gradient always first (bwd8w) / the data gradient always first
# (bwd8d) vs the longest-first rule
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in bwd8w bwd8d; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06bwd8o_$v ab/libpose6d_$v.so 2 || exit 1
done
