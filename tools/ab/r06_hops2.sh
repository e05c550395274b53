#!/bin/bash
# where the seeded ADD-S search's time goes: no-update builds with and without the seed walk
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06hops2}
mkdir -p $OUT
run() {  # label lib K
  POSE6D_LIB=${2:-} POSE6D_ADD_NEIGHBORS=$3 timeout -k 10 120 python -u tools/add_ab.py $OUT/$1.npz 2>/dev/null | sed "s/^/$1: /"
}
for r in 1 2 3; do
  run h2k16 ab/libpose6d_hops2.so 16 || exit 1
  run h2k16_noupdate ab/libpose6d_h2hit0.so 16 || exit 1
  run noseed_noupdate ab/libpose6d_h2hit0.so 0 || exit 1
done
