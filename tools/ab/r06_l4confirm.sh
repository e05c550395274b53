#!/bin/bash
# confirmation: layer4 3x3 bf16 weight gradients in one split (default) vs two (ab/libpose6d_l4twosplit.so); GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_lib.sh gpurun_out/r06l4confirm ab/libpose6d_l4twosplit.so 3 || exit 1
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py tests/test_config_parity.py tests/test_models.py tests/test_adamw_packed.py tests/test_checkpoint.py 2>&1 | tail -2
