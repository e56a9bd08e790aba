#!/bin/bash
# A/B of library builds on one box: for each .so in $LIBS (default: the in-tree build), optional parity tests ($TESTS
# with -k "$K") then the bench at one and four frames in flight ($STEPS timed steps), alternating builds twice.
# Output: gpurun_out/$1/<tag>_*.log and a summary line per run.  Each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5ab}
mkdir -p $O
export TMPDIR=/tmp
LIBS=${LIBS:-svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so}
STEPS=${STEPS:-40}
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps $STEPS --warmup 5 $BENCH_ARGS"
summ() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("stage_ms"), d["roofline"]["kernel"], d["roofline"]["avg_launch_ms"])'; }
for L in $LIBS; do
  t=$(basename $L .so)
  if [ -n "$TESTS" ]; then
    SVTGPU_LIB=$L timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread $TESTS -m gpu ${K:+-k "$K"} > $O/${t}_tests.log 2>&1 || { echo "$t tests failed"; tail -30 $O/${t}_tests.log; exit 1; }
    echo "$t: $(tail -1 $O/${t}_tests.log)"
  fi
done
for rep in 1 2; do
  for L in $LIBS; do
    t=$(basename $L .so)
    for F in ${FS:-1 4}; do
      SVTGPU_LIB=$L timeout -k 10 300 $B --frames-in-flight $F > $O/${t}_f${F}_$rep.log 2>&1 || { echo "$t bench F=$F failed"; tail -20 $O/${t}_f${F}_$rep.log; exit 1; }
      echo "$t F=$F rep $rep: $(summ $O/${t}_f${F}_$rep.log)"
    done
  done
done
echo done
