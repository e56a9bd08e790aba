#!/bin/bash
# gpu_r3_check_prof.sh (GPU tests matching $1, bench at F = 1 / 3, kernel traces) into gpurun_out/$2, then one short
# F = 1 bench with per-workgroup clocks (SVTGPU_WGCLK) into gpurun_out/$2/wg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r3_check_prof.sh "$1" "$2" || exit 1
O=gpurun_out/${2:-cp}/wg
mkdir -p $O
SVTGPU_WGCLK=$O/clk.bin timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --frames-in-flight 1 > $O/b.log 2>&1 || { echo "wgclk bench failed"; tail -5 $O/b.log; exit 1; }
echo wg done
