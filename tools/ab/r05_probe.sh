#!/bin/bash
# Round-5 probe: GPU suite, eval-forward per-layer times for each ab/ variant library,
# PMC passes over the eager eval forward.  usage: bash tools/ab/r05_probe.sh TAG [variants...]
TAG=${1:-r05b}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_base.txt 2>&1 || { tail $OUT/eval_base.txt; exit 1; }
head -1 $OUT/eval_base.txt
for v in "$@"; do
  POSE6D_LIB=ab/libpose6d_$v.so timeout -k 10 200 python -u tools/eval_layers.py 32 bf16 > $OUT/eval_$v.txt 2>&1 || { tail $OUT/eval_$v.txt; exit 1; }
  echo "$v: $(head -1 $OUT/eval_$v.txt)"
done
timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
if [ -n "$PMC" ]; then
  cd /tmp
  P=$GRAFT_REPO_ROOT/tools/eval_pmc.py
  i=0
  for G in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $G -d $GRAFT_REPO_ROOT/$OUT/pmc$i -o run --output-format csv -- python3 $P --reps 3 > $GRAFT_REPO_ROOT/$OUT/pmc$i.log 2>&1 || { echo "pmc pass $i rc=$?"; break; }
  done
  cd $GRAFT_REPO_ROOT
  REPS=3 python3 tools/eval_pmc_summary.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 > $OUT/pmc_summary.txt 2>&1
  rm -f $OUT/pmc*/*/*.csv.bak
  head -5 $OUT/pmc_summary.txt
fi
echo done
