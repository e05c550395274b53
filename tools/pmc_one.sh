#!/bin/bash
# PMC counter passes over tools/conv_bench.py for ONE conv shape and pass
# (one counter group per rocprofv3 run; kernel trace for durations).
# usage: tools/pmc_one.sh TAG SHAPE_INDEX PASS [bf16|f32]
TAG=$1; IDX=$2; PASS=$3; DT=${4:-bf16}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc1_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/tools/conv_bench.py --only $IDX --passes $PASS --impls fast --tiles auto --dtype $DT"
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
         "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- python3 $B > $OUT/p$i.log 2>&1 || echo "pass $i rc=$?" >> $OUT/fail.log
done
exit 0
