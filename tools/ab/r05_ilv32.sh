#!/bin/bash
# ILV on the fp32 (reference-precision) path: per-conv sweep and fp32 step A/B.
TAG=${1:-r05f}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/conv_bench.py --graph --dtype f32 --passes fwdns,dgrad --impls fast --tiles auto > $OUT/bench_base.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_bench.py --graph --dtype f32 --passes fwdns,dgrad --impls fast --tiles auto --lib ab/libpose6d_ilv.so > $OUT/bench_ilv.txt 2>&1 || exit 1
paste -d'\n' <(grep "|" $OUT/bench_base.txt) <(grep "|" $OUT/bench_ilv.txt | sed 's/^/ILV /')
bash tools/ab_lib.sh $OUT/ab_f32_ilv ab/libpose6d_ilv.so 3 fp32 || exit 1
echo done
