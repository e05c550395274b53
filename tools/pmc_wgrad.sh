#!/bin/bash
# SQ / TA / TCP / TCC counter passes on the bf16 weight-gradient kernel of single convs
# (tools/conv_one.py ... wgrad), one counter group per rocprofv3 run, + a kernel trace.
# usage: bash tools/pmc_wgrad.sh TAG
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcw_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/conv_one.py
i=0
for shape in "14 14 1024 256 1 1 0" "56 56 256 64 1 1 0" "14 14 256 256 3 1 1"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- python3 $P $shape wgrad 5 > $OUT/t$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $OUT/a$i -o run --output-format csv -- python3 $P $shape wgrad 5 > $OUT/a$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d $OUT/b$i -o run --output-format csv -- python3 $P $shape wgrad 5 > $OUT/b$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $OUT/c$i -o run --output-format csv -- python3 $P $shape wgrad 5 > $OUT/c$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum -d $OUT/d$i -o run --output-format csv -- python3 $P $shape wgrad 5 > $OUT/d$i.log 2>&1 || exit $?
done
exit 0
