#!/bin/bash
# F=3 A/B of environment settings (each arg a "NAME=VAL ..." list), two runs each, bench only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab3
i=0
for cfg in "$@"; do
  for k in 1 2; do
    env $cfg timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-matrix > gpurun_out/ab3/c${i}_$k.log 2>&1 || exit $?
    echo "[$cfg] $(grep '^{' gpurun_out/ab3/c${i}_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["frame_latency_ms"])')"
  done
  i=$((i+1))
done
