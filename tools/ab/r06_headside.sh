#!/bin/bash
# bf16 and fp32 steps: the head's Linear weight gradients on a side stream (POSE6D_HEAD_WGRAD_SIDE=1) vs on the step's
# stream (POSE6D_HEAD_WGRAD_SIDE=0), alternated on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06headside
mkdir -p $OUT
B="python bench.py --steps 40 --warmup 10 --no-side --no-fp32 --no-cpu-baseline --no-kernel-profile"
F="python tools/fp32_step.py"
for r in 1 2 3; do
  for cmd in B F; do
    POSE6D_HEAD_WGRAD_SIDE=1 timeout -k 10 200 ${!cmd} > $OUT/${cmd}_side_$r.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    POSE6D_HEAD_WGRAD_SIDE=0 timeout -k 10 200 ${!cmd} > $OUT/${cmd}_chain_$r.json 2>$OUT/err.txt || { tail $OUT/err.txt; exit 1; }
    python -c "
import json
a=json.load(open('$OUT/${cmd}_side_$r.json')); b=json.load(open('$OUT/${cmd}_chain_$r.json'))
print('round $r $cmd: side', a['ms_per_step'], 'chain', b['ms_per_step'], flush=True)"
  done
done
