#!/bin/bash
# Round-4 frames-in-flight sweep and an F = 4 kernel trace of the main loop only (no projection / matrix / CPU
# baseline), into gpurun_out/$1.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4sweep}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_f4 -o run --output-format csv -- $B --steps 40 --warmup 5 --frames-in-flight 4 > $O/trace_f4.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_f4.log; exit 1; }
for f in ${FS:-3 4 5 6}; do
  timeout -k 10 300 $B --steps 60 --warmup 5 --frames-in-flight $f > $O/b_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/b_f$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"])')"
done
echo done
