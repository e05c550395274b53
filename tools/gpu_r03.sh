#!/bin/bash
# round 3 box run: full GPU suite, bench (in-step roofline, fp32 line), optional library
# A/B, rocprofv3 kernel trace of the plain graph-replayed step.
# usage: bash tools/gpu_r03.sh TAG [VARIANT_SO]
set -o pipefail
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
echo bench ok
if [ -n "$2" ]; then bash tools/ab_lib.sh $OUT $2 3 || exit 1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline --no-fp32 --no-kernel-profile > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
echo prof ok
