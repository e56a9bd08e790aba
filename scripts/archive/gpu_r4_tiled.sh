#!/bin/bash
# Tiled-path tests (ranks on one GPU, RCCL one-rank, DLF device / host search) and the emulated 8-GPU rank, into
# gpurun_out/$1.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4tiled}
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
timeout -k 10 1000 $T tests/test_tiled_gpu.py tests/test_dlf_device_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 --warmup 5 --emulate-rank 8 > $O/e8.log 2>&1 || { echo "bench failed"; tail -20 $O/e8.log; exit 1; }
echo "E8 $(grep '^{' $O/e8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frames_in_flight"], c["frame_latency_ms"])')"
echo done
