#!/bin/bash
# in-step per-symbol breakdown (bench.py kernel_profile) for the default build and a variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r06i}; VAR=$2
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-side --no-fp32 --no-cpu-baseline > $OUT/base.json 2> $OUT/base.err || { tail $OUT/base.err; exit 1; }
POSE6D_LIB=$VAR timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-side --no-fp32 --no-cpu-baseline > $OUT/var.json 2> $OUT/var.err || { tail $OUT/var.err; exit 1; }
python - $OUT <<'PY'
import json, sys
d = sys.argv[1]
for n in ("base", "var"):
    r = json.loads(open(f"{d}/{n}.json").read().strip().splitlines()[-1])
    print(n, r["ms_per_step"], "eval", r["forward_roofline_eval"]["fwd_ms"])
    for k, v in list(r["breakdown"]["by_symbol"].items())[:14]:
        print(f"   {v['ms']*1000:8.1f} {v['launches']:3d} {v['avg_us']:7.2f} {k[:80]}")
PY
