cd $GRAFT_REPO_ROOT
for L in "" ab/libpose6d_nowp.so ab/libpose6d_nowt.so ab/libpose6d_nowpt.so; do
  echo "lib=${L:-default}"
  POSE6D_LIB=$L timeout -k 10 120 python -u tools/adamw_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
