#!/bin/bash
# configs[1] (PoseNetRGB bs32 fp32 eval, eager) kernel trace: last forward's launches,
# plus the bench with POSE6D_EVAL_DUAL_ROWS=0 (dual block launch on every stage)
OUT=$GRAFT_REPO_ROOT/gpurun_out/f32_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/t -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/rgb_fp32_once.py 5 > $OUT/log.txt 2>&1 || exit $?
CSV=$(ls $OUT/t/*/run_kernel_trace.csv $OUT/t/run_kernel_trace.csv 2>/dev/null | head -1)
python3 $GRAFT_REPO_ROOT/tools/trace_last.py $CSV 75 > $OUT/last.txt 2>&1
rm -rf $OUT/t
cd $GRAFT_REPO_ROOT
POSE6D_EVAL_DUAL_ROWS=0 timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_rows0.json 2> $OUT/bench.err
