#!/bin/bash
# host-side phase times of the LR search (SVTGPU_LR_TIMING) over a short F = 1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-lrt}
mkdir -p $O
SVTGPU_LR_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight 1 > $O/b.log 2> $O/err.log || { echo "bench failed"; tail -20 $O/err.log; exit 1; }
grep '^{' $O/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["frame_latency_ms"])'
grep 'lr_search ms' $O/err.log | tail -8
