#!/bin/bash
# After the fused DLF step counts every workgroup: the DLF / pipeline / async GPU tests, then the default-flag bench
# four times (whole frames, F = 4) and the emulated 8-GPU rank twice, with the DLF stage time per slot.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-dlf_arrival}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dlf_gpu.py tests/test_dlf_device_gpu.py tests/test_async_gpu.py tests/test_pipeline_golden.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection"
run() {
  timeout -k 10 240 python3 bench.py $B $2 > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  echo "$1: $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["concurrency"]["value"], c["concurrency"]["slot_latency_ms"], c["stage_ms"]["dlf_pick_filter"])')"
}
for r in 1 2 3 4; do run f4_r$r "--run-ahead 3"; done
for r in 1 2; do run e8_r$r "--emulate-rank 8"; done
