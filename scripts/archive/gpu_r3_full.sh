#!/bin/bash
# Round-end style check: the whole -m gpu suite, smoke(), the default bench (matrix included) and kernel traces at
# F = 1 / 4 (the default), into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None, {k: v.get("value") for k, v in d["config"].get("matrix", {}).items()} if isinstance(d["config"].get("matrix"), dict) else d["config"].get("matrix"))'
for f in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_f$f -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight $f > $O/trace_f$f.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_f$f.log; exit 1; }
done
echo done
