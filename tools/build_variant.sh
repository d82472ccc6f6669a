#!/bin/bash
# Build a diagnostics variant of libgx_amd.so with extra -D flags on one
# kernel source (timing experiments only; the GPU box selects it with GX_LIB):
#   tools/build_variant.sh NAME SOURCE "DEFINES"   e.g.  noplanes gx_fill_pk "-DGX_DIAG_NO_PLANES"
# (SOURCE: a csrc/*.hip or csrc/*.cpp file, without the extension)
set -e
cd "$(dirname "$0")/../genomics-rs_amd"
NAME=$1; SRC=$2; DEFS=$3
mkdir -p build_var
EXT=hip; [ -f csrc/$SRC.cpp ] && EXT=cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $DEFS -c -o build_var/$SRC.$NAME.o csrc/$SRC.$EXT
OBJS=$(ls build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o build_var/libgx_amd_$NAME.so $OBJS build_var/$SRC.$NAME.o
echo "built genomics-rs_amd/build_var/libgx_amd_$NAME.so"
