#!/bin/bash
# Emulated rank of an 8-GPU tiled picture with two builds (the in-tree library and $LIB), alternating twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5e8lib}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5 --emulate-rank ${N:-8}"
s() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("frame_latency_ms"), {k: round(v, 2) for k, v in c["stage_ms"].items() if k != "note"})'; }
for rep in 1 2; do
  for L in svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so $LIB; do
    t=$(basename $L .so)
    SVTGPU_LIB=$L timeout -k 10 300 $B > $O/${t}_$rep.log 2>&1 || { echo "$t failed"; tail $O/${t}_$rep.log; exit 1; }; echo "$t: $(s $O/${t}_$rep.log)"
  done
done
