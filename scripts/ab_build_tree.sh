#!/bin/bash
# Build the HIP extension of the WORKING TREE into OUTDIR, after applying an optional sed expression to
# common.h (timing experiments, e.g. plain stores in place of the fixed-point atomics):
#   SED='s/atomicAdd(reinterpret_cast<u64_t\*>(p), (u64_t)fx_q(v));/*p = fx_q(v);/' bash scripts/ab_build_tree.sh ab/plain
set -e
OUT=$1
SRC=$(mktemp -d)
cp -r self-replicating-artificial-neural-networks_amd/csrc/hip "$SRC/hip"
D=$SRC/hip
[ -n "$SED" ] && sed -i "$SED" "$D/common.h"
mkdir -p "$OUT"
SUF=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYI=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PBI=$(python3 -c "import pybind11;print(pybind11.get_include())")
for f in "$D"/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Wno-unused-result $ABFLAGS \
    -I"$D" -I"$PYI" -I"$PBI" -c "$f" -o "$SRC/$(basename "$f" .hip).o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 "$SRC"/*.o -o "$OUT/serann_hip$SUF"
rm -rf "$SRC"
echo "built $OUT/serann_hip$SUF"
