#!/bin/bash
# A/B of environment switches on one build: parity tests first, then SVTGPU_SR_STATS at one frame in flight and the
# bench at F = 1 / 4 for each variant.  Variants: VARS="name:ENV=1,ENV2=1 name2:..." (an empty env list is the
# default build); without VARS, "new:" against "old:$ENVAB".  Each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5srenv}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread $TESTS -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
VARS=${VARS:-"new: old:$ENVAB"}
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps ${STEPS:-30} --warmup 5"
for rep in $(seq 1 ${REPS:-2}); do
for VE in $VARS; do
  V=${VE%%:*}; E=${VE#*:}; E=${E//,/ }
  if [ -z "$NO_STATS" ]; then
  env $E SVTGPU_SR_STATS=1 SVTGPU_WR_STATS=1 timeout -k 10 300 $B --frames-in-flight 1 > $O/${V}_stats_$rep.log 2>&1 || { echo "$V stats failed"; tail -20 $O/${V}_stats_$rep.log; exit 1; }
  echo "$V stats: $(grep 'row-part' $O/${V}_stats_$rep.log | tail -1)"
  fi
  for F in 1 4; do
    env $E timeout -k 10 300 $B --frames-in-flight $F > $O/${V}_f${F}_$rep.log 2>&1 || { echo "$V F=$F failed"; tail -20 $O/${V}_f${F}_$rep.log; exit 1; }
    echo "$V F=$F: $(grep '^{' $O/${V}_f${F}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["config"]["stage_ms"]["'"${STAGE:-lr_search_apply}"'"], r["all_kernels_ms_per_frame"])')"
  done
done
done
echo done
