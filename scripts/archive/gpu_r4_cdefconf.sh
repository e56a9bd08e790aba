#!/bin/bash
# CDEF kernels: parity tests, LDS bank-conflict counters (one --pmc pass) and kernel durations (one --kernel-trace
# --stats pass), into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4cdefconf}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps ${PSTEPS:-4} --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing"
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_cdef_gpu.py tests/test_pipeline_golden.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-include-regex "${K:-cdef_search|cdef_apply}" -d $O/pmc -o run --output-format csv -- $B > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 60 > $O/b.log 2>&1 || { echo "bench failed"; tail -20 $O/b.log; exit 1; }
grep '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"]["cdef_search"])'
echo done
