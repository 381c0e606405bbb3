#!/bin/bash
# Build the HIP extension of the WORKING TREE with extra compile flags into OUTDIR (SERANN_NATIVE_DIR A/B runs of
# build-time knobs):  ABFLAGS="-DSERANN_DIVERGE_CHECK=0" bash scripts/ab_build_tree.sh ab/nochk
set -e
OUT=$1
D=self-replicating-artificial-neural-networks_amd/csrc/hip
TMP=$(mktemp -d)
mkdir -p "$OUT"
SUF=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYI=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PBI=$(python3 -c "import pybind11;print(pybind11.get_include())")
CC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Wno-unused-result $ABFLAGS -I$D -I$PYI -I$PBI"
for f in "$D"/*.hip; do
  b=$(basename "$f" .hip)
  if [ "$b" = gemm3 ]; then
    for p in 0 1 2 3; do $CC -DGEMM3_PART=$p -c "$f" -o "$TMP/${b}_p$p.o" & done
  elif [ "$b" = gchain ]; then
    $CC -mllvm -amdgpu-mfma-vgpr-form -c "$f" -o "$TMP/$b.o" &
  else
    $CC -c "$f" -o "$TMP/$b.o" &
  fi
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$TMP"/*.o -o "$OUT/serann_hip$SUF"
rm -rf "$TMP"
echo "built $OUT/serann_hip$SUF"
