#!/bin/bash
# confirmation: fp32 layer4 3x3 weight gradients in 2 splits (default now) vs the doubled target's 4 (ab/libpose6d_f32double.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_lib.sh gpurun_out/r06f32confirm ab/libpose6d_f32double.so 3 fp32 || exit 1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py tests/test_config_parity.py tests/test_models.py 2>&1 | tail -2
