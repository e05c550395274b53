#!/bin/bash
# eval-forward kernel traces (last graph replay) for two settings of one env variable
# usage: tools/gpu_evaltrace.sh TAG VAR VALUE_A VALUE_B
TAG=$1; VAR=$2; A=$3; B=$4
OUT=$GRAFT_REPO_ROOT/gpurun_out/evtrace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in $A $B; do
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t_$v -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/tools/eval_graph_once.py 20 > $OUT/log_$v.txt 2>&1 || exit $?
  CSV=$(ls $OUT/t_$v/*/run_kernel_trace.csv $OUT/t_$v/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 $GRAFT_REPO_ROOT/tools/trace_last.py $CSV 70 > $OUT/last_$v.txt 2>&1
  rm -rf $OUT/t_$v
done
