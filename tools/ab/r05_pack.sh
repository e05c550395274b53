#!/bin/bash
# AdamW-emits-packed-weights check: its tests + the trainer tests, A/B against the
# packing-pass layout (bf16 and fp32), kernel trace of the new step.
TAG=${1:-r05p}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_adamw_packed.py tests/test_config_parity.py tests/test_checkpoint.py tests/test_ddp_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_attr.py kw:pack_in_adamw --rounds 9 > $OUT/ab_bf16.txt 2>&1 || { tail $OUT/ab_bf16.txt; exit 1; }
cat $OUT/ab_bf16.txt
timeout -k 10 300 python -u tools/ab_attr.py kw:pack_in_adamw --rounds 7 --dtype f32 > $OUT/ab_f32.txt 2>&1 || { tail $OUT/ab_f32.txt; exit 1; }
cat $OUT/ab_f32.txt
bash tools/step_trace.sh $TAG || exit 1
grep -E "adamw|pack_kernel|sumsq" gpurun_out/trace_$TAG/window.txt
