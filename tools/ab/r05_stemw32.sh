#!/bin/bash
# fp32 row-tap stem weight gradient: conv / model tests, stem wgrad timing (row-tap
# LDS-DMA vs register-staged, split sweep), fp32 step time.
TAG=${1:-r05w32}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_conv_kernels.py tests/test_config_parity.py tests/test_models.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/conv_bench.py --dtype f32 --graph --only 0 --passes wgrad --tiles auto --wgrad-env "wgrad_base=1;wgrad_splits=32;wgrad_splits=64;wgrad_splits=128;wgrad_splits=256;wgrad_splits=512;wgrad_stages=3" > $OUT/stem_wgrad.txt 2>&1 || { tail $OUT/stem_wgrad.txt; exit 1; }
grep -v amdgpu.ids $OUT/stem_wgrad.txt
timeout -k 10 300 python -u tools/fp32_step.py > $OUT/fp32_step.json 2> $OUT/fp32_step.err || { tail $OUT/fp32_step.err; exit 1; }
cat $OUT/fp32_step.json
