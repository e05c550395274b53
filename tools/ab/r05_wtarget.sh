#!/bin/bash
# A/B of the bf16 weight-gradient split targets (build variants in ab/) on the step
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r05_wtarget
mkdir -p $OUT
for v in kxk512 kxk1024 all512; do
  echo "== $v"
  bash tools/ab_lib.sh $OUT/$v ab/libpose6d_$v.so 3 || exit 1
done
