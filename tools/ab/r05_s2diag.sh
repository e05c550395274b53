#!/bin/bash
# 1x1 stride-2 data gradients (the downsample convs): timing per pass and a kernel
# trace of the fp32 calls.
TAG=${1:-r05s2}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for dt in f32 bf16; do
  timeout -k 10 300 python -u tools/conv_bench.py --dtype $dt --graph --only 8,14,20,6,12 --passes fwd,dgrad,dgradip,bwd,bwdip --impls fast --tiles auto > $OUT/bench_$dt.txt 2>&1 || { tail $OUT/bench_$dt.txt; exit 1; }
  grep -v amdgpu.ids $OUT/bench_$dt.txt
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_bench.py --dtype f32 --only 8 --passes dgrad --impls fast --tiles auto > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200 | head -12
