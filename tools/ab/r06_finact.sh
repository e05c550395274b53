#!/bin/bash
# fused BN finalize + apply: bit-identity tests, then the attribute A/B (bf16 + fp32) and a breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06l}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bn_fusion.py \
  > $OUT/tests.log 2>&1 || { tail -50 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -2
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.bn_fused_finalize_act --rounds 5 > $OUT/ab_bf16.txt 2>&1 || { tail $OUT/ab_bf16.txt; exit 1; }
cat $OUT/ab_bf16.txt
timeout -k 10 300 python -u tools/ab_attr.py pose6d.trunk.TrunkEngine.bn_fused_finalize_act --rounds 3 --dtype f32 > $OUT/ab_f32.txt 2>&1 || { tail $OUT/ab_f32.txt; exit 1; }
cat $OUT/ab_f32.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-side --no-fp32 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - $OUT <<'PY'
import json, sys
r = json.loads(open(f"{sys.argv[1]}/bench.json").read().strip().splitlines()[-1])
print("step", r["ms_per_step"], "kernels", r["breakdown"]["kernels_per_step"], "eval", r["forward_roofline_eval"]["fwd_ms"])
for k, v in list(r["breakdown"]["by_symbol"].items())[:16]:
    print(f"   {v['ms']*1000:8.1f} {v['launches']:3d} {v['avg_us']:7.2f} {k[:80]}")
PY
