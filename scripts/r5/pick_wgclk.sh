#!/bin/bash
# Per-workgroup phase clocks of the CDEF pick steps (SVTGPU_WGCLK) on the bench's CDEF stages at one frame in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5pickclk}
mkdir -p $O
rm -f $O/clk.bin
SVTGPU_WGCLK=$O/clk.bin timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --stages cdef > $O/b.log 2>&1 || { echo "wgclk bench failed"; tail -5 $O/b.log; exit 1; }
python scripts/wgclk.py $O/clk.bin sod_step > $O/sod_step.txt && head -60 $O/sod_step.txt
