#!/bin/bash
# HIP runtime settings vs the replayed-graph launch floor (tools/launch_floor.py) and the bf16 step (bench.py, 40 steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/envfloor
mkdir -p $OUT
B="python bench.py --steps 40 --warmup 10 --no-side --no-fp32 --no-cpu-baseline --no-kernel-profile"
for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" \
         "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "AMD_DIRECT_DISPATCH=0" "X=0"; do
  echo "== $e"
  env $e timeout -k 10 120 python tools/launch_floor.py 2>/dev/null | grep -E "tiny|add" || exit 1
  env $e timeout -k 10 200 $B 2>/dev/null > $OUT/b.json || exit 1
  python -c "import json; print('bf16 step ms', json.load(open('$OUT/b.json'))['ms_per_step'])"
done
