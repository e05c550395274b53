#!/bin/bash
# ADD-S seed walk: hops (build) x neighbours per row K (POSE6D_ADD_NEIGHBORS), bit-compared
# against the round-6 in-order sweep; then the ADD GPU tests on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06hops}
mkdir -p $OUT
run() {  # label lib K
  POSE6D_LIB=${2:-} POSE6D_ADD_NEIGHBORS=$3 timeout -k 10 120 python -u tools/add_ab.py $OUT/$1.npz 2>/dev/null | sed "s/^/$1: /"
}
for r in 1 2 3; do
  run h3k32 "" 32 || exit 1
  run h3k16 "" 16 || exit 1
  run h1k32 ab/libpose6d_hops1.so 32 || exit 1
  run h2k16 ab/libpose6d_hops2.so 16 || exit 1
  run h2k32 ab/libpose6d_hops2.so 32 || exit 1
  run h5k16 ab/libpose6d_hops5.so 16 || exit 1
  run h5k8 ab/libpose6d_hops5.so 8 || exit 1
  run inorder ab/libpose6d_seed0.so 0 || exit 1
done
python - $OUT <<'PY'
import numpy as np, sys
d = sys.argv[1]
b = np.load(f"{d}/inorder.npz")
for t in ("h3k32", "h3k16", "h1k32", "h2k16", "h2k32", "h5k16", "h5k8"):
    a = np.load(f"{d}/{t}.npz")
    print(f"{t} == in-order sweep bit for bit:", all(np.array_equal(a[k], b[k]) for k in ("min", "argmin", "adds")))
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -3
