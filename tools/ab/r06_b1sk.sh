#!/bin/bash
# B = 1 inference with four K splits on small grids (default) vs the batch-32 rule only
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  TAG=small_grid_split4 timeout -k 10 200 python tools/inf_b1.py 2>/dev/null || exit 1
  TAG=batch32_rule_only POSE6D_LIB=ab/libpose6d_nosmallsk.so timeout -k 10 200 python tools/inf_b1.py 2>/dev/null || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_inference.py tests/test_conv_kernels.py 2>&1 | tail -2
