#!/bin/bash
# persistent CDEF pick phase ticks (SVTGPU_PICK_STATS, workgroup 0) over a short F = 1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pks}
mkdir -p $O
SVTGPU_PICK_STATS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-matrix --frames-in-flight 1 > $O/b.log 2> $O/err.log || { echo "bench failed"; tail -20 $O/err.log; exit 1; }
grep 'sod_persist' $O/err.log | tail -5
