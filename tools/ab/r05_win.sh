#!/bin/bash
# Fused-backward tile order: data-gradient tiles as interleaved streams per XCD
# (POSE6D_BWD_WIN variants).  Conv tests on one variant, step A/B, FETCH_SIZE per launch.
TAG=${1:-r05win}
VARS=${2:-"win1 win4 win16"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
first=${VARS%% *}
POSE6D_LIB=ab/libpose6d_$first.so timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in $VARS; do
  echo "== $v"
  bash tools/ab_lib.sh $OUT/$v ab/libpose6d_$v.so 2 || exit 1
done
bash tools/pmc_round.sh ${TAG}_base || exit 1
POSE6D_LIB=$GRAFT_REPO_ROOT/ab/libpose6d_$first.so bash tools/pmc_round.sh ${TAG}_$first || exit 1
head -4 gpurun_out/pmc_${TAG}_base/summary.txt
head -4 gpurun_out/pmc_${TAG}_$first/summary.txt
