#!/bin/bash
# Repeats of --run-ahead 2 and 3 at four frames (round 6 saw one 3 run collapse to 699 Mpx/s), with --host-timing so a
# collapse shows where the host waits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-runahead_rep}
mkdir -p $O
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --host-timing"
run() {
  timeout -k 10 240 python3 bench.py $B $2 > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  echo "$1: $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["concurrency"]["value"], c["concurrency"]["slot_latency_ms"])')"
}
for r in 1 2 3; do run ra3_r$r "--run-ahead 3"; run ra2_r$r "--run-ahead 2"; done
