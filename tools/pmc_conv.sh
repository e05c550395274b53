#!/bin/bash
# SQ counter passes on single conv kernels (tools/conv_one.py), one pass per group.
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcconv
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/conv_one.py
i=0
for shape in "7 7 512 512 3 1 1" "14 14 256 256 3 1 1" "56 56 64 64 3 1 1" "14 14 1024 256 1 1 0"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $OUT/a$i -o run --output-format csv -- python3 $P $shape fwd 3 > $OUT/a$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d $OUT/b$i -o run --output-format csv -- python3 $P $shape fwd 3 > $OUT/b$i.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $OUT/c$i -o run --output-format csv -- python3 $P $shape fwd 3 > $OUT/c$i.log 2>&1 || exit $?
done
