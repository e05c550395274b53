#!/bin/bash
# Kernel trace of replayed training steps + per-symbol / per-layer breakdowns.
# usage: tools/step_trace.sh TAG [extra step_profile args]
TAG=${1:-r}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/step_profile.py --steps 10 "$@" > $OUT/run.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
CSV=$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/trace_window.py $CSV --steps 10 --top 60 > $OUT/window.txt 2>&1
python3 tools/trace_layers.py $CSV > $OUT/layers.txt 2>&1
python3 tools/trace_seq.py $CSV > $OUT/seq.txt 2>&1
STATS=$(ls $OUT/*/run_kernel_stats.csv $OUT/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$STATS" ] && cp "$STATS" $OUT/kernel_stats.csv
rm -f $CSV
exit 0
