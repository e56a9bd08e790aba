#!/bin/bash
# Round-6 A/B of the frame-level modes on one box: the bench with the asynchronous DLF / LR searches and their
# synchronous forms ($MODES: lists of bench flags separated by ';'), at $FS frames in flight, $STEPS timed steps, with
# --host-timing.  Output: gpurun_out/$1/<i>_f<F>.log and one summary line per run.  Each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r6modes}
mkdir -p $O
export TMPDIR=/tmp
STEPS=${STEPS:-30}
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --host-timing --steps $STEPS --warmup 5 $BENCH_ARGS"
summ() { grep '^{' $1 | python -c '
import json,sys
d=json.loads(sys.stdin.read()); c=d["config"]
h=c.get("host_ms") or {}
print(d["value"], d["ms_per_step"], "lat", c.get("frame_latency_ms"), "conc", (c.get("concurrency") or {}).get("value"),
      {k: round(v, 3) for k, v in c["stage_ms"].items() if k != "note"}, c.get("dlf_search_mode"), json.dumps(h)[:400])'; }
IFS=';' read -ra ML <<< "${MODES:-;--dlf-sync;--lr-sync;--dlf-sync --lr-sync}"
i=0
for M in "${ML[@]}"; do
  for F in ${FS:-1 4}; do
    timeout -k 10 300 $B $M --frames-in-flight $F > $O/${i}_f${F}.log 2>&1 || { echo "bench [$M] F=$F failed"; tail -20 $O/${i}_f${F}.log; exit 1; }
    echo "[$M] F=$F: $(summ $O/${i}_f${F}.log)"
  done
  i=$((i+1))
done
echo done
