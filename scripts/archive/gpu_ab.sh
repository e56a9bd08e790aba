#!/bin/bash
# GPU parity tests, then the default bench with an environment switch on and off (A/B in the same box run).
# usage: gpu_ab.sh VAR  -> bench with VAR unset (A) and VAR=0 (B), F=1 and F=3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VAR=${1:-SVTGPU_SG_QUEUE}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest exit $rc"; exit $rc; }
for f in 1 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frames-in-flight $f > gpurun_out/bench_a_f$f.log 2>&1 || exit $?
  env $VAR=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frames-in-flight $f > gpurun_out/bench_b_f$f.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frames-in-flight $f > gpurun_out/bench_a2_f$f.log 2>&1 || exit $?
done
for x in gpurun_out/bench_*_f*.log; do echo "$x $(tail -1 $x | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["stage_ms"]["lr_search_apply"], d["config"].get("lr_search_kernel_ms"))')"; done
