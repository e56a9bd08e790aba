#!/bin/bash
# Builds experimental variants of the library (-DSGR_EXP=n) into scripts/ubench/var/ (dev tool).
set -e
cd "$(dirname "$0")/../../svt-av1_pro-anchor-v2.1.0-_amd"
mkdir -p ../scripts/ubench/var
for v in "$@"; do
  mkdir -p /tmp/var$v
  for f in csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -DSGR_EXP=$v -DDLF_EXP=$((v>>4)) -c $f -o /tmp/var$v/$(basename $f .hip).o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/var$v/*.o -o ../scripts/ubench/var/libsvtgpu_$v.so
done
