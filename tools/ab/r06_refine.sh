#!/bin/bash
# ADD-S: trip hits refined (strict test outside the trips before the best's) vs the seed
# walk without the refinement (ab/libpose6d_hops2.so) vs the round-6 in-order sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06refine}
mkdir -p $OUT
run() {  # label lib K
  POSE6D_LIB=${2:-} POSE6D_ADD_NEIGHBORS=$3 timeout -k 10 120 python -u tools/add_ab.py $OUT/$1.npz 2>/dev/null | sed "s/^/$1: /"
}
for r in 1 2 3; do
  run refine_h2k16 "" 16 || exit 1
  run refine_h2k32 "" 32 || exit 1
  run refine_h2k8 "" 8 || exit 1
  run refine_h3k16 ab/libpose6d_h3.so 16 || exit 1
  run refine_own_only "" 0 || exit 1
  run walk_h2k16_norefine ab/libpose6d_hops2.so 16 || exit 1
  run inorder ab/libpose6d_seed0.so 0 || exit 1
done
python - $OUT <<'PY'
import numpy as np, sys
d = sys.argv[1]
b = np.load(f"{d}/inorder.npz")
for t in ("refine_h2k16", "refine_h2k32", "refine_h2k8", "refine_h3k16", "refine_own_only", "walk_h2k16_norefine"):
    a = np.load(f"{d}/{t}.npz")
    print(f"{t} == in-order sweep bit for bit:", all(np.array_equal(a[k], b[k]) for k in ("min", "argmin", "adds")))
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -3
