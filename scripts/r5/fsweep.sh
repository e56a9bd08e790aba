#!/bin/bash
# Frames-in-flight sweep of the default bench (FS="3 5 6"), each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5fs}
mkdir -p $O
for F in ${FS:-3 5 6}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps ${STEPS:-40} --warmup 5 --frames-in-flight $F > $O/f$F.log 2>&1 || { echo "F=$F failed"; tail -20 $O/f$F.log; exit 1; }
  echo "F=$F: $(grep '^{' $O/f$F.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"].get("frame_latency_ms"))')"
done
