#!/bin/bash
# Round-end box run: full GPU suite, the default bench.py line (as the driver runs it),
# rocprofv3 kernel traces of the plain replayed bf16 and fp32 steps, the eval forward's
# per-launch times, the PMC traffic passes (bf16 and fp32) and the DDP overlap prediction.
# usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r06z}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo bench ok
bash tools/step_trace.sh ${TAG}_bf16 || exit 1
bash tools/step_trace.sh ${TAG}_f32 --dtype f32 || exit 1
echo traces ok
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_layers.txt 2> $OUT/eval_layers.err || { tail $OUT/eval_layers.err; exit 1; }
bash tools/pmc_round.sh ${TAG}_bf16 bf16 || exit 1
bash tools/pmc_round.sh ${TAG}_f32 f32 || exit 1
timeout -k 10 300 python tools/ddp_overlap.py --out $OUT/ddp_overlap_bf16.json > $OUT/ddp_overlap_bf16.log 2>&1 || exit 1
timeout -k 10 300 python tools/ddp_overlap.py --dtype f32 --out $OUT/ddp_overlap_f32.json > $OUT/ddp_overlap_f32.log 2>&1 || exit 1
echo done
