#!/bin/bash
# One environment setting over emulated ranks: "NAME=value:emu:F" entries (value '-' = unset; F '-' = the default),
# into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4envsweep}
mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in $CFGS; do
  IFS=: read kv e f <<< "$cfg"
  i=$((i+1))
  fa=""; [ "$f" != "-" ] && fa="--frames-in-flight $f"
  ev=""; [ "${kv#*=}" != "-" ] && ev="$kv"
  env $ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 --warmup 5 --emulate-rank $e $fa > $O/run$i.log 2>&1 || { echo "bench $cfg failed"; tail -20 $O/run$i.log; exit 1; }
  echo "$cfg $(grep '^{' $O/run$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; s=c["stage_ms"]; print(d["value"], c["frames_in_flight"], c["frame_latency_ms"], {k: v for k, v in s.items() if k != "note"})')"
done
echo done
