#!/bin/bash
# Self-guided search diagnostics at one frame in flight (SVTGPU_SR_STATS) and the VALU issue microbenchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4stats}
mkdir -p $O
[ -n "$ALU" ] && { timeout -k 10 60 scripts/ubench/alu > $O/alu.log 2>&1 || { echo "alu failed"; exit 1; }; }
[ -n "$ALU" ] && cat $O/alu.log
SVTGPU_WR_STATS=1 SVTGPU_SR_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing > $O/stats.log 2>&1 || { echo "stats failed"; tail -20 $O/stats.log; exit 1; }
grep -E "sgr_res|wiener_res" $O/stats.log | tail -2
