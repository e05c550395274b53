#!/bin/bash
# round 4: pipelined conv K loop -- microbench, conv parity, per-shape timing, A/B vs the unpipelined build
O=$GRAFT_REPO_ROOT/gpurun_out/pipe
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/ldsdma_spec_bench > $O/spec.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_kernels.py tests/test_inference.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --graph --passes fwd,dgrad,bwd --tiles auto --stages auto --impls fast > $O/conv_pipe.txt 2>&1 || exit $?
POSE6D_LIB=ab/libpose6d_nopipe.so timeout -k 10 300 python tools/conv_bench.py --graph --passes fwd,dgrad,bwd --tiles auto --stages auto --impls fast > $O/conv_nopipe.txt 2>&1 || exit $?
bash tools/ab_lib.sh $O/ab_eval ab/libpose6d_nopipe.so 3 eval > $O/ab_eval.txt 2>&1 || exit $?
bash tools/ab_lib.sh $O/ab_bf16 ab/libpose6d_nopipe.so 3 > $O/ab_bf16.txt 2>&1 || exit $?
bash tools/ab_lib.sh $O/ab_fp32 ab/libpose6d_nopipe.so 2 fp32 > $O/ab_fp32.txt 2>&1 || exit $?
