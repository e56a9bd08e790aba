#!/bin/bash
# frames-in-flight sweep of the default bench (no CPU baseline, no matrix), two runs each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/inflight
for f in ${@:-2 3 4 5 6}; do
  for k in 1 2; do
    timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --no-matrix --frames-in-flight $f > gpurun_out/inflight/f${f}_$k.log 2>&1 || exit $?
    echo "F=$f run $k $(grep '^{' gpurun_out/inflight/f${f}_$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["frame_latency_ms"])')"
  done
done
