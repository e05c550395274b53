#!/bin/bash
# the seeded ADD-S search (default build, K = 16 / 0) vs the round-6 start's kernel
# (ab/libpose6d_r06y_add.so, add_eval.hip at ad01302) on one box: bench.py's own
# configs[3] timing and tools/add_ab.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06addcmp; mkdir -p $OUT
for r in 1 2 3; do
  TAG=seeded_k16 timeout -k 10 120 python tools/add_bench_side.py 2>/dev/null || exit 1
  TAG=no_table_k0 POSE6D_ADD_NEIGHBORS=0 timeout -k 10 120 python tools/add_bench_side.py 2>/dev/null || exit 1
  TAG=r06y_kernel POSE6D_ADD_NEIGHBORS=0 POSE6D_LIB=ab/libpose6d_r06y_add.so timeout -k 10 120 python tools/add_bench_side.py 2>/dev/null || exit 1
done
for r in 1 2; do
  timeout -k 10 120 python tools/add_ab.py $OUT/a.npz 2>/dev/null | sed "s/^/add_ab seeded_k16: /" || exit 1
  POSE6D_ADD_NEIGHBORS=0 POSE6D_LIB=ab/libpose6d_r06y_add.so timeout -k 10 120 python tools/add_ab.py $OUT/b.npz 2>/dev/null | sed "s/^/add_ab r06y_kernel: /" || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -2
