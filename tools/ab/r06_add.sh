#!/bin/bash
# ADD points-kernel variants: timing + bit-identity across variants, then the ADD tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06_add}
mkdir -p $OUT
for v in 1 2 3 4 5 6 0; do
  POSE6D_ADD_VARIANT=$v timeout -k 10 120 python -u tools/add_ab.py $OUT/v$v.npz || exit 1
done
python - $OUT <<'PY'
import numpy as np, sys, glob
d = sys.argv[1]
ref = np.load(f"{d}/v1.npz")
for f in sorted(glob.glob(f"{d}/v*.npz")):
    x = np.load(f)
    print(f, all(np.array_equal(x[k], ref[k]) for k in ("min", "argmin", "adds")))
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_add_loss.py 2>&1 | tail -3
