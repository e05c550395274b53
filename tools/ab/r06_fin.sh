#!/bin/bash
# training BN finalize: one-wave fold (<= 512 rows, default) vs the whole-workgroup fold for
# every row count (ab/libpose6d_finall256.so): isolated launches, then the bf16 / fp32 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06fin}
mkdir -p $OUT
echo "== base (wave fold <= 512 rows)"; timeout -k 10 120 python tools/fin_bench.py 2>/dev/null || exit 1
echo "== all rows whole-workgroup fold"; POSE6D_LIB=ab/libpose6d_finall256.so timeout -k 10 120 python tools/fin_bench.py 2>/dev/null || exit 1
echo "== bf16 step"; bash tools/ab_lib.sh $OUT/bf16 ab/libpose6d_finall256.so 3 || exit 1
echo "== fp32 step"; bash tools/ab_lib.sh $OUT/f32 ab/libpose6d_finall256.so 2 fp32 || exit 1
