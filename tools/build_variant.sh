#!/bin/bash
# Build an A/B variant of libpose6d.so with compile-time definitions on some sources:
#   bash tools/build_variant.sh NAME "-DPOSE6D_BN_FOLD_ROWS=0" bn.hip [more.hip ...]
# -> ab/libpose6d_NAME.so (the other objects from the regular build); select it at run
# time with POSE6D_LIB=ab/libpose6d_NAME.so (pose6d/_lib.py).
set -e
NAME=$1; DEFS=$2; shift 2
REPO=$(cd "$(dirname "$0")/.." && pwd)
SRC=$REPO/6d-pose-estimation_amd/csrc
make -C "$SRC" -s -j8
mkdir -p "$REPO/ab/obj_$NAME"
objs=""
for f in "$SRC"/*.hip; do
  b=$(basename "$f" .hip)
  if [[ " $* " == *" $b.hip "* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -I"$REPO/include" -I"$SRC" -Wall \
      -Wno-unused-function $DEFS -c "$f" -o "$REPO/ab/obj_$NAME/$b.o"
    objs="$objs $REPO/ab/obj_$NAME/$b.o"
  else
    objs="$objs $SRC/build/$b.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$REPO/ab/libpose6d_$NAME.so" $objs
echo "built ab/libpose6d_$NAME.so"
