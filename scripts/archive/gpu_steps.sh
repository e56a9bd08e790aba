#!/bin/bash
# Run-to-run spread of the headline line against the timed-step count (three frames in flight).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/steps
for n in 20 100 20 100 20 100; do
  timeout -k 10 300 python bench.py --steps $n --warmup 5 --no-cpu-baseline --no-matrix > gpurun_out/steps/s$n.log 2>&1 || exit $?
  echo "steps $n $(tail -1 gpurun_out/steps/s$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
