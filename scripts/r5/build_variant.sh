#!/bin/bash
# An experiment build of the library (CPU, here): lr_search.hip recompiled with extra defines, linked with the other
# in-tree objects into lib_exp/libsvtgpu_<name>.so (git-ignored; loaded through SVTGPU_LIB by scripts/r5/ab_lib.sh).
#   bash scripts/r5/build_variant.sh sr1024 -DSVTGPU_SR_NT=1024
set -e
cd "$(dirname "$0")/../../svt-av1_pro-anchor-v2.1.0-_amd"
name=$1; shift
make -s lib/libsvtgpu.so
mkdir -p lib_exp build_exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics "$@" \
    -c csrc/lr_search.hip -o build_exp/lr_search_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v lr_search.o) build_exp/lr_search_$name.o \
    -o lib_exp/libsvtgpu_$name.so -L/opt/rocm/lib -lrccl
echo "lib_exp/libsvtgpu_$name.so"
