#!/bin/bash
# Kernel-trace statistics (rocprofv3 --kernel-trace --stats) of short one-frame-in-flight bench runs in the given
# mode(s) ($MODES: bench flag lists separated by ';'), into gpurun_out/$1/m<i>/.  Each run under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r6prof}
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra ML <<< "${MODES:-;--dlf-sync}"
i=0
for M in "${ML[@]}"; do
  mkdir -p $O/m$i
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/m$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-matrix \
      --no-tile-projection --no-kernel-timing --steps ${STEPS:-10} --warmup 3 --frames-in-flight ${F:-1} $M \
      > $O/m$i/bench.log 2>&1 || { echo "profile [$M] failed"; tail -20 $O/m$i/bench.log; exit 1; }
  f=$(find $O/m$i -name '*kernel_stats.csv' | head -1)
  echo "[$M] $(grep '^{' $O/m$i/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["stage_ms"]["dlf_pick_filter"])')"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("  %-70s calls %6s avg %9.1f us total %8.2f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                           float(r["TotalDurationNs"]) / 1e6))
PY
  i=$((i+1))
done
echo done
