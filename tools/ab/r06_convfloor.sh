#!/bin/bash
# conv launch floor: the eval-forward conv (BN + ReLU epilogue) at batch 1 / 2 / 8 / 32 for a 1x1 and a 3x3 shape
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for B in 1 2 8 32; do
  echo "B=$B"; timeout -k 10 120 python tools/conv_bench.py --graph --B $B --only 21,22,15,16 --passes fwdact,fwdns --tiles auto --impls fast 2>/dev/null || exit 1
done
