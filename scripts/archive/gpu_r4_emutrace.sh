#!/bin/bash
# Kernel trace of one emulated rank of the 8-GPU tiled picture (bench --emulate-rank 8) at four frames in flight,
# into gpurun_out/$1; then the same without the trace for the figures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4emu}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --emulate-rank 8"
timeout -k 10 300 $B --steps 40 --warmup 5 --host-timing > $O/b_e8.log 2>&1 || { echo "bench failed"; tail -20 $O/b_e8.log; exit 1; }
grep '^{' $O/b_e8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"], c.get("host_timing"))'
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- $B --steps 20 --warmup 3 > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
echo done
