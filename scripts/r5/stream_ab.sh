#!/bin/bash
# Streaming-kernel A/B of library builds ($LIBS): FETCH_SIZE and WRITE_SIZE passes (separate) and a kernel trace of the
# bench at one frame in flight per build; scripts/r5/stream_summary.py prints bytes and duration per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5stream}
mkdir -p $O
export TMPDIR=/tmp
K="cdef_apply|lr_apply|dlf_tile|md_dist"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing --lr-serial"
for L in $LIBS; do
  t=$(basename $L .so)
  export SVTGPU_LIB=$L
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/${t}_fetch -o run --output-format csv -- $B > $O/${t}_fetch.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/${t}_write -o run --output-format csv -- $B > $O/${t}_write.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${t}_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --lr-serial > $O/${t}_trace.log 2>&1 || { echo "$t failed"; exit 1; }
  python3 scripts/r5/stream_summary.py $O $t
done
