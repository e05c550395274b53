#!/bin/bash
# A/B of two library builds on one box, alternating: bash tools/ab_lib.sh OUTDIR VARIANT_SO [rounds] [fp32]
# (bench.py bf16 training step, or with "fp32" the fused fp32 step of tools/fp32_step.py;
# the default build is "base")
OUT=$1; VAR=$2; ROUNDS=${3:-3}
CMD="python bench.py --steps 40 --warmup 10 --no-side --no-fp32 --no-cpu-baseline --no-kernel-profile"
[ "${4:-}" = "fp32" ] && CMD="python tools/fp32_step.py"
[ "${4:-}" = "eval" ] && CMD="python tools/eval_time.py"
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  timeout -k 10 200 $CMD > $OUT/ab_base_$r.json 2>/dev/null || exit 1
  POSE6D_LIB=$VAR timeout -k 10 200 $CMD > $OUT/ab_var_$r.json 2>/dev/null || exit 1
  python -c "
import json,sys
a=json.load(open('$OUT/ab_base_$r.json')); b=json.load(open('$OUT/ab_var_$r.json'))
print('round $r: base', a['ms_per_step'], 'variant', b['ms_per_step'], flush=True)"
done
