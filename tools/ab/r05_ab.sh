#!/bin/bash
# GPU suite (patch tests first), eval per-layer times (new vs ab/libpose6d_old.so), A/B of
# the bf16 training step and of the eval forward.  usage: bash tools/ab/r05_ab.sh TAG [rounds]
TAG=${1:-r05c}; R=${2:-3}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "patch or fast_variants or splitk" > $OUT/tests_patch.log 2>&1 || { tail -40 $OUT/tests_patch.log; exit 1; }
tail -1 $OUT/tests_patch.log
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_new.txt 2>&1 || { tail $OUT/eval_new.txt; exit 1; }
POSE6D_LIB=ab/libpose6d_old.so timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_old.txt 2>&1 || exit 1
grep "^# eval" $OUT/eval_new.txt $OUT/eval_old.txt
bash tools/ab_lib.sh $OUT/ab_eval ab/libpose6d_old.so $R eval || exit 1
bash tools/ab_lib.sh $OUT/ab_step ab/libpose6d_old.so $R || exit 1
echo done
