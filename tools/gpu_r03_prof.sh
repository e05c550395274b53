#!/bin/bash
# round 3 profiling box run: PMC passes (bf16 and fp32 steps), drop-in fp32 host/GPU
# profile, eval-forward per-launch times.  usage: bash tools/gpu_r03_prof.sh TAG
set -o pipefail
TAG=${1:-r03p}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_layers.txt 2> $OUT/eval_layers.err || { tail $OUT/eval_layers.err; exit 1; }
timeout -k 10 200 python -u tools/dropin_profile.py --steps 10 > $OUT/dropin.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/dropin_prof -o run -- python3 tools/dropin_profile.py --steps 10 --markers > $OUT/dropin_prof.log 2>&1 || exit 1
python tools/dropin_profile.py --analyze $OUT/dropin_prof --steps 10 >> $OUT/dropin.txt 2>&1
bash tools/pmc_round.sh ${TAG}_bf16 bf16 || exit 1
bash tools/pmc_round.sh ${TAG}_f32 f32 || exit 1
echo done
