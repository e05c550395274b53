#!/bin/bash
# ADD min-test variants; 8-wave fused backward: conv tests, teacher-forced bs32 test, step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06g}
mkdir -p $OUT
for v in 5 10 11 12 14; do
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
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py \
  tests/test_config_parity.py tests/test_bn_fusion.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_lib.sh $OUT/ab ab/libpose6d_nobf128.so 3 || exit 1
