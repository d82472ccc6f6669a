#!/bin/bash
# Mutation check of the overlapped two-group pipeline's stream order
# (gx_api_batch.cpp batch_core_overlap): builds gpurun_exp/nowait/libgx_amd.so
# from the current objects with gx_api_batch.cpp's
#     HIPCHK(hipStreamWaitEvent(sB, ctx->slots[a].te, 0));
# removed (step k+1's group-B fill then no longer waits for step k's walk,
# which still reads B's plane codes).  Run on the GPU, once:
#     GX_LIB=gpurun_exp/nowait/libgx_amd.so python -m pytest -m gpu \
#         tests/test_gpu_atsize.py -k overlapped_alternating_sets
# must FAIL (tests/test_gpu_atsize.py test_overlapped_alternating_sets);
# the normal library passes it.  Needs `make` run first (the other objects).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)/genomics-rs_amd
D=$(cd "$(dirname "$0")/.." && pwd)/gpurun_exp/nowait
mkdir -p "$D"
sed '/HIPCHK(hipStreamWaitEvent(sB, ctx->slots\[a\].te, 0));/d' "$R/csrc/gx_api_batch.cpp" > "$D/gx_api_batch.cpp"
if cmp -s "$R/csrc/gx_api_batch.cpp" "$D/gx_api_batch.cpp"; then echo "mutation: line not found" >&2; exit 1; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I"$R/csrc" \
    -c -o "$D/gx_api_batch.o" "$D/gx_api_batch.cpp"
OBJS=$(ls "$R"/build/*.o | grep -v '/gx_api_batch.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$D/libgx_amd.so" $OBJS "$D/gx_api_batch.o"
rm -f "$D/gx_api_batch.o"
echo "built $D/libgx_amd.so (overlap wait removed)"
