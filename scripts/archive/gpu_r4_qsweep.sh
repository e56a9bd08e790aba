#!/bin/bash
# Hardware-queue sweep: "emu:F:queues" triples (emu 1 = the whole frame), into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4qsweep}
mkdir -p $O
export TMPDIR=/tmp
for cfg in $CFGS; do
  IFS=: read e f q <<< "$cfg"
  SVTGPU_BENCH_QUEUES=$q timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 --warmup 5 --emulate-rank $e --frames-in-flight $f > $O/e${e}_f${f}_q$q.log 2>&1 || { echo "bench $cfg failed"; tail -20 $O/e${e}_f${f}_q$q.log; exit 1; }
  echo "$cfg $(grep '^{' $O/e${e}_f${f}_q$q.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["stage_ms"]; print(d["value"], c["frame_latency_ms"], {k: v for k, v in s.items() if k != "note"})')"
done
echo done
