#!/bin/bash
# Self-guided search diagnostics: SVTGPU_SR_STATS per search (one-part vs row-part items) at one frame in flight,
# then the bench line with the event-timed roofline.  Each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5srstats}
mkdir -p $O
export TMPDIR=/tmp
SVTGPU_SR_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 10 --warmup 2 --frames-in-flight 1 > $O/srstats.log 2>&1 || { echo "srstats failed"; tail -20 $O/srstats.log; exit 1; }
grep "sgr_res:" $O/srstats.log | tail -4
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_ms"], r["avg_launch_ms_device_clock"], r["frac"])'
echo done
