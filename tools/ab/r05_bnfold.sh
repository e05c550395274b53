#!/bin/bash
# In-launch BN finalize (pose6d_conv2d_fwd_bn): its tests, the trainer parity tests,
# A/B of TrunkEngine.bn_fold_fwd on the bf16 / fp32 steps, kernel trace of the step.
TAG=${1:-r05f}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_conv_kernels.py tests/test_bn_fusion.py tests/test_adamw_packed.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bn_fold or splitk or bn_fusion or dual or trainer or packed or configs2" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.bn_fold_fwd --rounds 9 > $OUT/ab_bf16.txt 2>&1 || { tail $OUT/ab_bf16.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_bf16.txt
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.bn_fold_fwd --rounds 7 --dtype f32 > $OUT/ab_f32.txt 2>&1 || { tail $OUT/ab_f32.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_f32.txt
bash tools/step_trace.sh $TAG || exit 1
head -30 gpurun_out/trace_$TAG/window.txt
