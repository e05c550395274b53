#!/bin/bash
# Exploration pass on the GPU box: fp32 forward tile sweep (8-wave tiles included),
# eval-forward kernel trace (last graph replay), training-step kernel trace.
# usage: tools/gpu_explore.sh TAG
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/explore_$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/conv_bench.py --graph --dtype f32 --passes fwd --impls fast --tiles auto,3,4,5 \
  --stages auto,2,3 > $OUT/f32_tiles.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/evtrace -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/eval_graph_once.py 20 > $OUT/evtrace.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
CSV=$(ls $OUT/evtrace/*/run_kernel_trace.csv $OUT/evtrace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_last.py $CSV 70 > $OUT/eval_last.txt 2>&1
rm -f $CSV
bash tools/step_trace.sh $TAG
