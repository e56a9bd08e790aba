#!/bin/bash
# Emulated rank of an 8-GPU tiled picture: the bounded exchange waits (default) against SVTGPU_COMM_WAIT=sync, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5e8}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5 --emulate-rank ${N:-8}"
s() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("frame_latency_ms"), {k: round(v, 2) for k, v in c["stage_ms"].items() if k != "note"})'; }
for rep in 1 2; do
  timeout -k 10 300 $B > $O/def_$rep.log 2>&1 || { echo "default failed"; tail $O/def_$rep.log; exit 1; }; echo "default: $(s $O/def_$rep.log)"
  SVTGPU_COMM_WAIT=sync timeout -k 10 300 $B > $O/sync_$rep.log 2>&1 || { echo "sync failed"; exit 1; }; echo "sync:    $(s $O/sync_$rep.log)"
done
