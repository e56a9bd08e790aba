#!/bin/bash
# Faster iteration: GPU tests matching $1 (pytest -k), a short bench and a kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K="${1:-gpu}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
