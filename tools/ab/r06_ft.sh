#!/bin/bash
# fp32 step: workgroup target of the fp32 128x128 (KxK) weight-gradient plans: 192 / 128 / 384 vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in ft192 ft128 ft384; do
  echo "== base vs $v"; bash tools/ab_lib.sh gpurun_out/r06ft_$v ab/libpose6d_$v.so 2 fp32 || exit 1
done
