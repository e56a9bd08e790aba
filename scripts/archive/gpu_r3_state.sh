#!/bin/bash
# Round-3 state check: the whole GPU suite, smoke, the default bench (cpu baseline + matrix) and one frame in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/state
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-600
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight 1 > $O/bench_f1.log 2>&1 || { echo "bench f1 failed"; tail -20 $O/bench_f1.log; exit 1; }
grep '^{' $O/bench_f1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("F=1", d["value"], c["frame_latency_ms"], c["stage_ms"])'
