#!/bin/bash
# Timing experiments on layout 3 (gx_skew.hip GX_SKEW_EXP bits; results are
# WRONG in every variant but 0): build one libgx_amd.so per variant into
# genomics-rs_amd/exp/, then time them on the GPU with
#     GX_LIB=genomics-rs_amd/exp/libgx_amd_expN.so SKEW_DIAG_QUICK=1 python tools/skew_diag.py 2
#   bit 1: no column-symbol loads; 2: no core -> side hand-off (side idle);
#   4: no ring reads / input waits; 8: no pushes to the strip below.
# (Measured, a lone 64 x 30,000 strip, traced ns/step: full 61.7; 1: 60.8;
# 4: 62.3; 2: 52.4; 8: 53.5; 2+8: 43.5; 1+2+4+8: 42.5.)
set -e
cd "$(dirname "$0")/../genomics-rs_amd"
make -s libgx_amd.so
mkdir -p exp
OBJS="build/gx_kernels.o build/gx_fill_pk.o build/gx_cs2.o build/gx_wide.o build/gx_api.o build/gx_host.o"
for v in "$@"; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DGX_SKEW_EXP=$v -c -o exp/gx_skew_$v.o csrc/gx_skew.hip
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o exp/libgx_amd_exp$v.so $OBJS exp/gx_skew_$v.o
    rm exp/gx_skew_$v.o
done
