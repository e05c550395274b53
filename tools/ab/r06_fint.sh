#!/bin/bash
# what the BN finalize launches cost inside the bf16 step: timing-only builds where the
# finalize kernels return at entry (fint1: the launch alone) or are not launched (fint2)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06fint; mkdir -p $OUT
echo "== base vs finalize kernels empty"; bash tools/ab_lib.sh $OUT/t1 ab/libpose6d_fint1.so 3 || exit 1
echo "== base vs finalize not launched"; bash tools/ab_lib.sh $OUT/t2 ab/libpose6d_fint2.so 3 || exit 1
