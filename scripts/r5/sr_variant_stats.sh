#!/bin/bash
# SVTGPU_SR_STATS of an experiment build (LIB, via SVTGPU_LIB) and of the in-tree build, one frame in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5srvar}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 20 --warmup 3 --frames-in-flight 1"
for L in svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so $LIB; do
  t=$(basename $L .so)
  SVTGPU_LIB=$L SVTGPU_SR_STATS=1 timeout -k 10 300 $B > $O/$t.log 2>&1 || { echo "$t failed"; tail -20 $O/$t.log; exit 1; }
  echo "$t: $(grep 'sgr_res:' $O/$t.log | tail -2 | tr '\n' ' ')"
done
