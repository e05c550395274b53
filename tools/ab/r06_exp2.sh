#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06f}
mkdir -p $OUT
for v in 5 3 4 6 7 9; do
  POSE6D_ADD_VARIANT=$v timeout -k 10 120 python -u tools/add_ab.py $OUT/v$v.npz || exit 1
done
python - $OUT <<'PY'
import numpy as np, sys, glob
d = sys.argv[1]
ref = np.load(f"{d}/v5.npz")
for f in sorted(glob.glob(f"{d}/v*.npz")):
    x = np.load(f)
    print(f, all(np.array_equal(x[k], ref[k]) for k in ("min", "argmin", "adds")))
PY
timeout -k 10 600 python -u tools/conv_bench.py --graph --passes wgrad --only 6,10,12,16,18,22,5,11,17 \
  --wgrad-env "wgrad_base=4;wgrad_base=4,wgrad_splits=16;wgrad_base=4,wgrad_splits=32;wgrad_base=4,wgrad_stages=4;wgrad_base=4,wgrad_splits=16,wgrad_stages=3;wgrad_splits=16" > $OUT/wgrad128_sweep2.txt 2>&1 || { tail -20 $OUT/wgrad128_sweep2.txt; exit 1; }
cat $OUT/wgrad128_sweep2.txt
