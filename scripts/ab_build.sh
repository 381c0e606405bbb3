#!/bin/bash
# Build the HIP extension of git revision REF into OUTDIR (for SERANN_NATIVE_DIR A/B timing runs).
#   bash scripts/ab_build.sh HEAD ab/prev
set -e
REF=$1; OUT=$2
SRC=$(mktemp -d)
git archive "$REF" self-replicating-artificial-neural-networks_amd/csrc/hip | tar -x -C "$SRC"
D=$SRC/self-replicating-artificial-neural-networks_amd/csrc/hip
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
