#!/bin/bash
# Round-6 GPU check: selected -m gpu tests ($TESTS, default: the whole suite), optionally smoke, then the default
# bench, into gpurun_out/$1.  Every GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r6check}
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 250 --timeout-method thread"
timeout -k 10 1000 $T ${TESTS:-tests} -m gpu ${K:+-k "$K"} > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
if [ -n "$SMOKE" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
timeout -k 10 900 python bench.py $BENCH_ARGS > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)'
fi
echo done
