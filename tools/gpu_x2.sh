#!/bin/bash
# in-graph vs hot conv durations in the eval forward; eval epilogue cost per conv shape
OUT=$GRAFT_REPO_ROOT/gpurun_out/x2
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/conv_bench.py --graph --passes fwdns,fwdact,fwdactres --impls fast --tiles auto \
  --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 > $OUT/act.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/dup -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/eval_dup_trace.py 10 > $OUT/dup.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
CSV=$(ls $OUT/dup/*/run_kernel_trace.csv $OUT/dup/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_last.py $CSV 125 > $OUT/dup_last.txt 2>&1
rm -f $CSV
