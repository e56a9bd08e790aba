#!/bin/bash
# GPU parity tests only (optionally a -k expression as $1): one pytest process, per-test timeout, log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
args=(tests -m gpu -x -v --timeout 300 --timeout-method thread)
[ -n "$1" ] && args+=(-k "$1")
timeout -k 10 900 python -u -m pytest "${args[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "exit $rc"
exit $rc
