#!/bin/bash
# round-6 experiment 1: ADD variants; bf16 128x128 8-wave weight gradient (check + sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06e}
mkdir -p $OUT
for v in 1 2 5 8 3 4 7; do
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
timeout -k 10 300 python -u tools/wgrad128_check.py > $OUT/wgrad128_check.txt 2>&1 || { tail -20 $OUT/wgrad128_check.txt; exit 1; }
tail -3 $OUT/wgrad128_check.txt
timeout -k 10 600 python -u tools/conv_bench.py --graph --passes wgrad --only 5,7,9,10,11,12,13,14,15,16,17,18,19,20,21,22 \
  --wgrad-env "wgrad_base=4;wgrad_base=4,wgrad_stages=3" > $OUT/wgrad128_sweep.txt 2>&1 || { tail -20 $OUT/wgrad128_sweep.txt; exit 1; }
cat $OUT/wgrad128_sweep.txt
