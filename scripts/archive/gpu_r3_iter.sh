#!/bin/bash
# Round-3 iteration: GPU tests matching $1 (pytest -k), then the default bench and one frame in flight, each with the
# environment settings given as the remaining args ("NAME=VAL ..." per configuration; "" = defaults).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/it
export TMPDIR=/tmp
K="${1:-gpu}"
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" \
    > gpurun_out/it/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/it/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/it/pytest.log | tail -1
i=0
for cfg in "$@"; do
  for f in 1 3; do
    env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix \
        --frames-in-flight $f > gpurun_out/it/b${i}_f$f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/it/b${i}_f$f.log; exit 1; }
    echo "[$cfg] F=$f $(grep '^{' gpurun_out/it/b${i}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"]["lr_search_apply"], c["lr_search_kernel_ms"])')"
  done
  i=$((i+1))
done
