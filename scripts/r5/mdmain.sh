#!/bin/bash
# The MD batch on the main stream (--md-main: one hardware queue less per frame) with more frames in flight:
# the emulated 8-GPU rank at F = 6 (default) / 7 / 8, then the whole frame at F = 4 / 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5mdm}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5"
s() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("frame_latency_ms"), {k: round(v, 2) for k, v in c["stage_ms"].items() if k != "note"})'; }
run() { n=$1; shift; timeout -k 10 300 $B "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail $O/$n.log; exit 1; }; echo "$n: $(s $O/$n.log)"; }
run e8_f6 --emulate-rank 8
run e8_f6_mdm --emulate-rank 8 --md-main
run e8_f7_mdm --emulate-rank 8 --md-main --frames-in-flight 7
run e8_f8_mdm --emulate-rank 8 --md-main --frames-in-flight 8
run f4 --frames-in-flight 4
run f4_mdm --frames-in-flight 4 --md-main
run f5_mdm --frames-in-flight 5 --md-main
