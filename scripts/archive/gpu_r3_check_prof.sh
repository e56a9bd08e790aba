#!/bin/bash
# GPU tests matching $1, the bench at F = 1 / 3, then rocprofv3 --kernel-trace --stats of the bench at F = 1 and 3
# (per-kernel device time of the current build) into gpurun_out/$2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${2:-cp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$1" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for f in 1 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight $f > $O/b_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/b_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"])')"
done
for f in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_f$f -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight $f > $O/trace_f$f.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_f$f.log; exit 1; }
done
echo done
