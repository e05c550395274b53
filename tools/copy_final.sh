#!/bin/bash
# copy a tools/ab/r06_final.sh run's outputs from gpurun_out/ into profiles/ (TAG_*)
T=${1:?tag}
set -e
cp gpurun_out/$T/bench.json profiles/${T}_bench.json
cp gpurun_out/$T/tests.log profiles/${T}_gpu_tests.log
cp gpurun_out/trace_${T}_bf16/window.txt profiles/${T}_step_trace.txt
cp gpurun_out/trace_${T}_bf16/layers.txt profiles/${T}_step_layers.txt
cp gpurun_out/trace_${T}_bf16/kernel_stats.csv profiles/${T}_kernel_stats.csv
cp gpurun_out/trace_${T}_f32/window.txt profiles/${T}_f32_step_trace.txt
cp gpurun_out/trace_${T}_f32/layers.txt profiles/${T}_f32_step_layers.txt
cp gpurun_out/trace_${T}_f32/kernel_stats.csv profiles/${T}_f32_kernel_stats.csv
cp gpurun_out/$T/eval_layers.txt profiles/${T}_eval_layers.txt
cp gpurun_out/pmc_${T}_bf16/pmc.json profiles/${T}_pmc.json
cp gpurun_out/pmc_${T}_bf16/summary.txt profiles/${T}_pmc_summary.txt
cp gpurun_out/pmc_${T}_f32/pmc.json profiles/${T}_f32_pmc.json
cp gpurun_out/pmc_${T}_f32/summary.txt profiles/${T}_f32_pmc_summary.txt
cp gpurun_out/$T/ddp_overlap_bf16.json profiles/${T}_ddp_overlap_bf16.json
cp gpurun_out/$T/ddp_overlap_f32.json profiles/${T}_ddp_overlap_f32.json
echo copied $T
