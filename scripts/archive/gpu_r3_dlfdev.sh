#!/bin/bash
# The device-resident DLF level search: its GPU tests (single rank at chunks 6 / 2 / 4, two tiled ranks), then an A/B
# of the default bench (host-driven vs device-resident search) at one and four frames in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-dlfdev}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dlf_device_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for f in 1 4; do
  for m in 0 1; do
    SVTGPU_DLF_DEVICE=$m timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-matrix --frames-in-flight $f > $O/bench_f${f}_d$m.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_f${f}_d$m.log; exit 1; }
    echo "F=$f dev=$m $(grep '^{' $O/bench_f${f}_d$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["frame_latency_ms"], d["config"]["stage_ms"])')"
  done
done
echo done
