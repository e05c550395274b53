#!/bin/bash
# Row-tap stem on the LDS-DMA path: conv / pack / trainer tests, stem plan sweep,
# eval-forward layers, A/B-free step numbers (bench) and a step trace.
TAG=${1:-r05s}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_conv_kernels.py tests/test_adamw_packed.py tests/test_models.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/conv_bench.py --graph --only 0 --passes fwd,fwdnst --tiles auto,1,3 --stages auto,2,3,4 > $OUT/stem_bf16.txt 2>&1 || { tail $OUT/stem_bf16.txt; exit 1; }
grep -v amdgpu.ids $OUT/stem_bf16.txt
timeout -k 10 300 python -u tools/conv_bench.py --graph --only 0 --passes fwd,fwdnst --tiles auto,1,3 --stages auto,2,3,4 --dtype f32 > $OUT/stem_f32.txt 2>&1 || { tail $OUT/stem_f32.txt; exit 1; }
grep -v amdgpu.ids $OUT/stem_f32.txt
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_layers.txt 2>&1 || { tail $OUT/eval_layers.txt; exit 1; }
head -6 $OUT/eval_layers.txt
bash tools/step_trace.sh $TAG || exit 1
head -3 gpurun_out/trace_$TAG/window.txt; grep -E "conv_lds_kernel<[^>]*6, |ILi6E|conv_igemm_kernel|wgrad_kernel" gpurun_out/trace_$TAG/window.txt | head
