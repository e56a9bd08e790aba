#!/bin/bash
# config 1 (1080p 8-bit CDEF search + pick + apply, one frame in flight): three bench runs and a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-c1}
mkdir -p $O
export TMPDIR=/tmp
C1="--width 1920 --height 1080 --bit-depth 8 --stages cdef --no-cpu-baseline --no-matrix --steps 100 --warmup 5 --frames-in-flight 1"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $C1 > $O/b$i.log 2>&1 || { echo "bench failed"; tail -20 $O/b$i.log; exit 1; }
  echo "run $i $(grep '^{' $O/b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["stage_ms"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $C1 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
