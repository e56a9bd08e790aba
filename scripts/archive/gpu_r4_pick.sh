#!/bin/bash
# Round-4 CDEF pick check: the CDEF and pipeline GPU tests, then the bench at F = 1 under rocprofv3 kernel stats and
# at F = 4, into gpurun_out/$1.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4pick}
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 250 --timeout-method thread"
timeout -k 10 600 $T tests/test_cdef_gpu.py tests/test_pipeline_golden.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_f1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 > $O/trace_f1.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_f1.log; exit 1; }
for f in 1 4; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight $f > $O/b_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/b_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"])')"
done
echo done
if [ -n "$EMU" ]; then
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-matrix --no-tile-projection --emulate-rank 8 > $O/b_e8.log 2>&1 || { echo "emulated bench failed"; tail -20 $O/b_e8.log; exit 1; }
  echo "E8 $(grep '^{' $O/b_e8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"])')"
fi
