#!/bin/bash
# Build a variant of the in-tree HIP extension with gchain.hip compiled under extra flags, linked
# with the other in-tree objects (serann/_build), into ab/NAME (for SERANN_NATIVE_DIR A/B runs).
# SRC=path builds another copy of gchain.hip (e.g. the committed one, from git show).
#   bash scripts/ab_gchain.sh NAME "-DGC_BWD_MINW=2"
set -e
NAME=$1; FLAGS=$2
D=self-replicating-artificial-neural-networks_amd
OUT=ab/$NAME; mkdir -p $OUT
SUF=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYI=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PBI=$(python3 -c "import pybind11;print(pybind11.get_include())")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Wno-unused-result $FLAGS \
  -mllvm -amdgpu-mfma-vgpr-form -I$D/csrc/hip -I"$PYI" -I"$PBI" -I$D/csrc/hip -c ${SRC:-$D/csrc/hip/gchain.hip} -o $OUT/gchain.o
objs=$(ls $D/_build/*.o | grep -v gchain.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $OUT/gchain.o -o $OUT/serann_hip$SUF
rm $OUT/gchain.o
echo "built $OUT/serann_hip$SUF"
