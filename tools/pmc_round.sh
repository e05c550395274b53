#!/bin/bash
# PMC passes (one counter group per run, never combined with trace domains):
# HBM read / write bytes and MFMA busy cycles per kernel of the eager training step.
# usage: tools/pmc_round.sh TAG [bf16|f32]
TAG=${1:-r}
DT=${2:-bf16}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/step_profile.py
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $P --eager --steps 2 --dtype $DT > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $P --eager --steps 2 --dtype $DT > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/mfma -o run --output-format csv -- python3 $P --eager --steps 2 --dtype $DT > $OUT/mfma.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py $OUT/pmc.json $OUT/fetch $OUT/write $OUT/mfma > $OUT/summary.txt 2>&1
