#!/bin/bash
# Frames in flight x the MD batch's stream (its own, or --md-main: one hardware queue less per frame) for whole frames
# and for the emulated 8-GPU rank (bench --emulate-rank 8); one bench process per point, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-fsweep_md}
mkdir -p $O
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection"
run() { # name, args
  timeout -k 10 240 python3 bench.py $B $2 > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  echo "$1: $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("concurrency",{}).get("value", c.get("concurrency")))')"
}
run f4 "--frames-in-flight 4"
run f4_mdmain "--frames-in-flight 4 --md-main"
run f5_mdmain "--frames-in-flight 5 --md-main"
run f6_mdmain "--frames-in-flight 6 --md-main"
run e8_f6 "--emulate-rank 8 --frames-in-flight 6"
run e8_f6_mdmain "--emulate-rank 8 --frames-in-flight 6 --md-main"
run e8_f7_mdmain "--emulate-rank 8 --frames-in-flight 7 --md-main"
run e8_f8_mdmain "--emulate-rank 8 --frames-in-flight 8 --md-main"
