#!/bin/bash
# Conv-level diagnostics of the 3x3 forwards: graph-timed ring-depth sweep of the patch
# kernel against the implicit GEMM, then PMC passes (one counter group per run) on the
# layer3 and layer4 3x3 shapes.  usage: bash tools/ab/r05_convdiag.sh TAG
TAG=${1:-r05d}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/conv_bench.py --graph --passes fwdnst --only 2,10,16,22 \
  --env "conv_patch=0;conv_patch=1,conv_stages=2;conv_patch=1,conv_stages=3;conv_patch=1,conv_stages=6;conv_patch=1,conv_stages=8" \
  > $OUT/sweep.txt 2>&1 || { tail $OUT/sweep.txt; exit 1; }
cat $OUT/sweep.txt | grep -v amdgpu.ids
cd /tmp
for IDX in 16 22; do
  i=0
  for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/pmc_$IDX/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_bench.py --only $IDX --passes fwdnst --env "conv_patch=0" > $OUT/pmc_${IDX}_p$i.log 2>&1 || echo "pmc $IDX pass $i rc=$?"
  done
  cd $GRAFT_REPO_ROOT
  python3 tools/pmc1_sum.py $OUT/pmc_$IDX > $OUT/pmc_${IDX}_summary.txt 2>&1
  rm -rf $OUT/pmc_$IDX
  cd /tmp
done
cd $GRAFT_REPO_ROOT
grep -A40 "patch\|conv_lds_kernel" $OUT/pmc_16_summary.txt | head -90
echo done
