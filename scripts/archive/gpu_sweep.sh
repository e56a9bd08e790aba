#!/bin/bash
# Parity tests of the changed stages, then bench runs over an environment sweep: SWEEP="VAR=a VAR=b ...".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K="${1:-gpu}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for kv in $SWEEP; do
  echo "== $kv" >> gpurun_out/sweep.log
  env "$kv" timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/sweep.log 2>&1 || exit 1
done
echo "exit 0"
