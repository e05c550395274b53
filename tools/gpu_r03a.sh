#!/bin/bash
# round 3, first box: head fix + eval teacher-forced + augment tests, bench with in-step timing,
# rocprof trace of the plain step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_augment.py tests/test_head_kernels.py tests/test_inference.py tests/test_crop.py "tests/test_config_parity.py::test_configs2_eval_forward_bs32_bf16_teacher_forced" > gpurun_out/r03a/tests.log 2>&1 || { tail -40 gpurun_out/r03a/tests.log; exit 1; }
tail -2 gpurun_out/r03a/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { tail -30 gpurun_out/r03a/bench.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03a/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline --no-fp32 --no-kernel-profile > gpurun_out/r03a/prof.log 2>&1 || { tail -30 gpurun_out/r03a/prof.log; exit 1; }
echo prof ok
