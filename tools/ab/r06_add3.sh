#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06m}
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 120 python -u tools/add_ab.py $OUT/hit2.npz | sed "s/^/hit2 (one step per point): /" || exit 1
  POSE6D_LIB=ab/libpose6d_addhit1.so timeout -k 10 120 python -u tools/add_ab.py $OUT/hit1.npz | sed "s/^/hit1 (in-order updates): /" || exit 1
  POSE6D_LIB=ab/libpose6d_addhit0.so timeout -k 10 120 python -u tools/add_ab.py $OUT/hit0.npz | sed "s/^/hit0 (timing only, no updates): /" || exit 1
done
python - $OUT <<'PY'
import numpy as np, sys
d = sys.argv[1]
a, b = np.load(f"{d}/hit2.npz"), np.load(f"{d}/hit1.npz")
print("hit2 == hit1:", all(np.array_equal(a[k], b[k]) for k in ("min", "argmin", "adds")))
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -1
