#!/bin/bash
# Row-tap stem weight gradient: conv / trainer / parity tests, stem wgrad timing
# (row-tap LDS-DMA vs the register-staged kernel), A/B-free step trace.
TAG=${1:-r05w}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_conv_kernels.py tests/test_adamw_packed.py tests/test_config_parity.py tests/test_checkpoint.py tests/test_models.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/conv_bench.py --graph --only 0 --passes wgrad,fwd --tiles auto --wgrad-env "wgrad_base=1" > $OUT/stem_wgrad.txt 2>&1 || { tail $OUT/stem_wgrad.txt; exit 1; }
grep -v amdgpu.ids $OUT/stem_wgrad.txt
bash tools/step_trace.sh $TAG || exit 1
head -3 gpurun_out/trace_$TAG/window.txt; grep -E "wgrad_lds_kernel|conv_wgrad_kernel|ILi6E|Li6ELi2" gpurun_out/trace_$TAG/window.txt | head
timeout -k 10 300 python -u bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['fp32_train']['ms_per_step'],d['forward_roofline_eval']['fwd_ms'])"
