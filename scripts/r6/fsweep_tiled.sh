#!/bin/bash
# Emulated tiled ranks (bench --emulate-rank N, N = 2 / 4 / 8) at six and seven frames in flight, two runs each:
# the choice of bench.py's TILED_FRAMES_IN_FLIGHT.  One bench process per point, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-fsweep_tiled}
mkdir -p $O
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection"
for rep in 1 2; do
  for n in 8 4 2; do
    for f in 6 7; do
      L=$O/e${n}_f${f}_r$rep.log
      timeout -k 10 240 python3 bench.py $B --emulate-rank $n --frames-in-flight $f > $L 2>&1 || { echo "e$n f$f failed"; tail -5 $L; exit 1; }
      echo "e$n f$f r$rep: $(grep '^{' $L | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["concurrency"]["value"], c["concurrency"]["streams_per_frame"])')"
    done
  done
done
