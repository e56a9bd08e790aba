#!/bin/bash
# Emulated 8-GPU rank with one stream per frame in flight (the LR search's Wiener chain after its self-guided chain on
# the frame's stream: --lr-serial with the Wiener stream never made, SVTGPU_LR_WST_LAZY=1; the MD batch on the main
# stream), so more frames fit the 16 hardware queues; against the default two streams at F = 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-fsweep_one}
mkdir -p $O
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --emulate-rank ${N:-8}"
run() {
  timeout -k 10 240 env $3 python3 bench.py $B $2 > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  echo "$1: $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["concurrency"]["value"])')"
}
run f7 "--frames-in-flight 7" ""
run f7_one "--frames-in-flight 7 --lr-serial --md-main" "SVTGPU_LR_WST_LAZY=1"
run f9_one "--frames-in-flight 9 --lr-serial --md-main" "SVTGPU_LR_WST_LAZY=1"
run f11_one "--frames-in-flight 11 --lr-serial --md-main" "SVTGPU_LR_WST_LAZY=1"
run f13_one "--frames-in-flight 13 --lr-serial --md-main" "SVTGPU_LR_WST_LAZY=1"
