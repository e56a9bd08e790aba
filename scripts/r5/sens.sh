#!/bin/bash
# Sensitivity runs (diagnostic): the default bench at four frames in flight with parts of the LR search switched off
# ($LVLS: wn,sg pairs), to see what each chain costs the throughput.  Each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5sens}
mkdir -p $O
export TMPDIR=/tmp
for L in ${LVLS:-1,1 0,1 1,0 0,0}; do
  for F in ${FS:-4 1}; do
    t=lr${L/,/_}_f$F
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps ${STEPS:-30} --warmup 5 --frames-in-flight $F --lr-levels $L $BENCH_ARGS > $O/$t.log 2>&1 || { echo "$t failed"; tail -20 $O/$t.log; exit 1; }
    echo "$t: $(grep '^{' $O/$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("stage_ms"))')"
  done
done
echo done
