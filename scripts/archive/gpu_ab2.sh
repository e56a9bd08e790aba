#!/bin/bash
# GPU parity tests, then the bench under several environment settings (each a "NAME=VAL ..." word list), F=1 and F=3.
# usage: gpu_ab2.sh "" "SVTGPU_WN_UNIT=0" "SVTGPU_WN_NG=2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest exit $rc"; exit $rc; }
i=0
for cfg in "$@"; do
  for f in 1 3; do
    env $cfg timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --no-matrix --frames-in-flight $f > gpurun_out/ab_${i}_f$f.log 2>&1 || exit $?
    echo "[$cfg] F=$f $(tail -1 gpurun_out/ab_${i}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["stage_ms"]["lr_search_apply"], d["config"].get("lr_search_kernel_ms"))')"
  done
  i=$((i+1))
done
