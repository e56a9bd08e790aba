#!/bin/bash
# Emulated ranks of tiled pictures (bench.py --emulate-rank N) across frames in flight: is the N-GPU step bound by
# device work, by replicated work or by the host?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4emu}
mkdir -p $O
for cfg in "8 4" "8 8" "8 12" "4 4" "4 8" "1 8"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --emulate-rank $1 --frames-in-flight $2 --host-timing > $O/emu_$1_$2.log 2>&1 || { echo "emu $cfg failed"; tail -20 $O/emu_$1_$2.log; exit 1; }
  echo "N=$1 F=$2 $(grep '^{' $O/emu_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["frame_latency_ms"], c["stage_ms"]["cdef_pick_apply"], c["stage_ms"]["lr_search_apply"], c["stage_ms"]["dlf_pick_filter"], c.get("host_ms"))')"
done
