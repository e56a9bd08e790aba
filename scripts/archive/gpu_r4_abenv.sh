#!/bin/bash
# A/B of one environment setting over the bench at F = 1, F = 4 (twice) and the emulated 8-GPU rank, alternating
# A and B, into gpurun_out/$1.  usage: VAR=NAME A=valueA B=valueB gpu_r4_abenv.sh <out>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4abenv}
mkdir -p $O
export TMPDIR=/tmp
B0="python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 --warmup 5"
run() { # tag value args
  env $VAR=$2 timeout -k 10 300 $B0 ${@:3} > $O/$1.log 2>&1 || { echo "bench $1 failed"; tail -20 $O/$1.log; exit 1; }
  echo "$1 $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["stage_ms"]; print(d["value"], c["frame_latency_ms"], s["cdef_pick_apply"], s["lr_search_apply"])')"
}
for r in 1 2; do
  run A_f4_$r "$A" --frames-in-flight 4
  run B_f4_$r "$B" --frames-in-flight 4
done
run A_f1 "$A" --frames-in-flight 1
run B_f1 "$B" --frames-in-flight 1
run A_e8 "$A" --emulate-rank 8
run B_e8 "$B" --emulate-rank 8
echo done
