#!/bin/bash
# Frames-in-flight sweep of the emulated 8-GPU rank (bench --emulate-rank 8), into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4e8sweep}
mkdir -p $O
export TMPDIR=/tmp
for f in ${FS:-3 5 6}; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 --warmup 5 --emulate-rank ${EMU:-8} --frames-in-flight $f > $O/e8_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/e8_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/e8_f$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["stage_ms"]; print(d["value"], c["frame_latency_ms"], {k: v for k, v in s.items() if k != "note"})')"
done
echo done
