#!/bin/bash
# round-end box run: full GPU suite, the default bench.py line (as the driver runs it),
# rocprofv3 kernel trace of the plain replayed step, eval-forward per-launch times and
# the PMC traffic passes [, an eval-forward A/B against VARIANT_SO].
# usage: bash tools/gpu_r03_final.sh TAG [VARIANT_SO]
set -o pipefail
TAG=${1:-r03f}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline --no-fp32 --no-kernel-profile > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo prof ok
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_layers.txt 2> $OUT/eval_layers.err || { tail $OUT/eval_layers.err; exit 1; }
bash tools/pmc_round.sh ${TAG}_bf16 bf16 || exit 1
if [ -n "$2" ]; then bash tools/ab_lib.sh $OUT/ab_eval $2 3 eval || exit 1; fi
echo done
