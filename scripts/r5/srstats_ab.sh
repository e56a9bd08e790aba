#!/bin/bash
# SVTGPU_SR_STATS for each library build in $LIBS at one frame in flight (diagnostic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5srab}
mkdir -p $O
export TMPDIR=/tmp
for L in $LIBS; do
  t=$(basename $L .so)
  SVTGPU_LIB=$L SVTGPU_SR_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 10 --warmup 2 --frames-in-flight 1 > $O/$t.log 2>&1 || { echo "$t failed"; tail -20 $O/$t.log; exit 1; }
  echo "$t: $(grep '^{' $O/$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["stage_ms"]["lr_search_apply"])')"
  grep "sgr_res:" $O/$t.log | tail -2
done
echo done
