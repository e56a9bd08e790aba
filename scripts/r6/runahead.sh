#!/bin/bash
# --run-ahead K (steps a frame slot's thread may enqueue ahead of its stream) for whole frames (F = 4) and the
# emulated 8-GPU rank (F = 7); one bench process per point, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-runahead}
mkdir -p $O
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection"
run() {
  timeout -k 10 240 python3 bench.py $B $2 > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  echo "$1: $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["concurrency"]["value"])')"
}
for k in 1 2 3 4; do run f4_ra$k "--run-ahead $k"; done
for k in 2 3 4; do run e8_ra$k "--emulate-rank 8 --run-ahead $k"; done
