#!/bin/bash
# ILV (DMA interleaved with MFMAs) variant: correctness, per-conv sweep, eval layers, step A/B.
TAG=${1:-r05e}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
POSE6D_LIB=ab/libpose6d_ilv.so timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py tests/test_inference.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_ilv.log 2>&1 || { tail -40 $OUT/tests_ilv.log; exit 1; }
tail -1 $OUT/tests_ilv.log
timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py tests/test_inference.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_base.log 2>&1 || { tail -40 $OUT/tests_base.log; exit 1; }
tail -1 $OUT/tests_base.log
timeout -k 10 300 python -u tools/conv_bench.py --graph --passes fwdns,dgrad --impls fast --tiles auto > $OUT/bench_base.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --graph --passes fwdns,dgrad --impls fast --tiles auto --lib ab/libpose6d_ilv.so > $OUT/bench_ilv.txt 2>&1 || exit 1
paste -d'\n' <(grep "|" $OUT/bench_base.txt) <(grep "|" $OUT/bench_ilv.txt | sed 's/^/ILV /')
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_new.txt 2>&1 || exit 1
POSE6D_LIB=ab/libpose6d_ilv.so timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_ilv.txt 2>&1 || exit 1
POSE6D_LIB=ab/libpose6d_old.so timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_old.txt 2>&1 || exit 1
grep "^# eval" $OUT/eval_*.txt
bash tools/ab_lib.sh $OUT/ab_step_ilv ab/libpose6d_ilv.so 3 || exit 1
bash tools/ab_lib.sh $OUT/ab_eval_old ab/libpose6d_old.so 2 eval || exit 1
echo done
