#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py \
  tests/test_config_parity.py tests/test_models.py tests/test_bn_fusion.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/ab_lib.sh $OUT/ab ab/libpose6d_nofuse128.so 3 fp32 || exit 1
