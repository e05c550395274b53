#!/bin/bash
# ADD-S search seeds: own ground-truth point + K model-space neighbours (default build,
# POSE6D_ADD_NEIGHBORS = K) vs the round-6 in-order sweep (ab/libpose6d_seed0.so) and the
# no-update timing floor; bit-compared; then the ADD GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06seed}
mkdir -p $OUT
for r in 1 2 3; do
  for K in 32 16 8 0; do
    POSE6D_ADD_NEIGHBORS=$K timeout -k 10 120 python -u tools/add_ab.py $OUT/k$K.npz 2>/dev/null | sed "s/^/seeds own+K=$K: /" || exit 1
  done
  POSE6D_LIB=ab/libpose6d_seed0.so timeout -k 10 120 python -u tools/add_ab.py $OUT/seed0.npz 2>/dev/null | sed "s/^/round-6 in-order sweep (no seeds): /" || exit 1
done
POSE6D_LIB=ab/libpose6d_seed1hit0.so POSE6D_ADD_NEIGHBORS=0 timeout -k 10 120 python -u tools/add_ab.py $OUT/hit0.npz 2>/dev/null | sed "s/^/timing floor (no updates): /" || exit 1
python - $OUT <<'PY'
import numpy as np, sys
d = sys.argv[1]
b = np.load(f"{d}/seed0.npz")
for K in (32, 16, 8, 0):
    a = np.load(f"{d}/k{K}.npz")
    print(f"K={K} == in-order sweep bit for bit:", {k: bool(np.array_equal(a[k], b[k])) for k in ("min", "argmin", "adds")})
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -3
