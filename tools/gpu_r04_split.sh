#!/bin/bash
# round 4: default split-K rule + fp32 LDS-DMA weight gradient -- parity, timing
O=$GRAFT_REPO_ROOT/gpurun_out/split
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_kernels.py tests/test_inference.py tests/test_config_parity.py tests/test_models.py -m gpu > $O/tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/fp32_step.py > $O/fp32_step.json 2>&1 || exit $?
timeout -k 10 200 python tools/eval_time.py > $O/eval.json 2>&1 || exit $?
timeout -k 10 300 python tools/conv_bench.py --graph --dtype f32 --passes wgrad,fwd,dgrad --env 'conv_splitk=2;conv_splitk=4;conv_tile=4;conv_tile=4,conv_splitk=2' --wgrad-env 'wgrad_stages=3;wgrad_base=1' > $O/f32_sweep.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-side --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 120 tools/ldsdma_spec_bench > $O/spec4.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ddp_overlap.py --out $O/ddp_overlap_bf16.json > $O/ddp_overlap.log 2>&1 || exit $?
bash tools/pmc_one.sh f32fwd3x3 2 fwd f32 && python3 tools/pmc1_sum.py gpurun_out/pmc1_f32fwd3x3 conv_lds > $O/pmc_f32fwd3x3.txt 2>&1
bash tools/pmc_one.sh bf16fwd1x1 15 fwd bf16 && python3 tools/pmc1_sum.py gpurun_out/pmc1_bf16fwd1x1 conv_lds > $O/pmc_bf16fwd1x1.txt 2>&1
