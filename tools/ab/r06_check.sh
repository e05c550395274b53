#!/bin/bash
# Round-6 GPU check: the tests this round touched first (verbose), then the whole GPU
# suite, then the default bench line.  usage: bash tools/ab/r06_check.sh TAG [--no-bench]
set -o pipefail
TAG=${1:-r06a}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_config_parity.py tests/test_models.py::test_bf16_trunk_odd_width_row_tap_stem \
  tests/test_adamw_packed.py tests/test_ddp_gpu.py::test_rccl_world1_bucketed_step > $OUT/new_tests.log 2>&1 \
  || { tail -60 $OUT/new_tests.log; exit 1; }
tail -3 $OUT/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
[ "$2" == "--no-bench" ] && exit 0
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo bench ok
python - $OUT/bench.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", r["value"], "ms", r["ms_per_step"], "frac", r["roofline"]["frac"], r["roofline"]["kernel"], r["roofline"]["avg_launch_us"])
print("fp32", r["fp32_train"]["ms_per_step"], r["fp32_train"]["roofline"]["frac"], "eval", r["forward_roofline_eval"]["fwd_ms"], r["forward_roofline_eval"]["frac"])
print("add", r["side_configs"]["configs[3]"]["ms_per_batch"], "cpu", r["cpu_baseline"])
PY
