#!/bin/bash
# CDEF pick partition sweep (SVTGPU_PICK_PARTS): F=1 bench stage times per setting into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pp}
mkdir -p $O
for p in 8 16 32 64; do
  SVTGPU_PICK_PARTS=$p timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight 1 > $O/b_p$p.log 2>&1 || { echo "bench failed p=$p"; tail -20 $O/b_p$p.log; exit 1; }
  echo "parts=$p $(grep '^{' $O/b_p$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["stage_ms"]["cdef_pick_apply"])')"
done
