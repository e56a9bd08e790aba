#!/bin/bash
# A/B of an environment switch (default vs "$AB", e.g. SVTGPU_SR_XCH=l2): parity of both, the self-guided diagnostics
# and the bench at one and four frames in flight, into gpurun_out/$1.  Each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4ab}
mkdir -p $O
T="python -u -m pytest -x -q --timeout 250 --timeout-method thread"
timeout -k 10 600 $T tests/test_lr_gpu.py tests/test_pipeline_golden.py tests/test_lr_modes_gpu.py -m gpu > $O/pytest_a.log 2>&1 || { echo "pytest A failed"; tail -30 $O/pytest_a.log; exit 1; }
tail -1 $O/pytest_a.log
env $AB timeout -k 10 600 $T tests/test_pipeline_golden.py tests/test_lr_gpu.py -m gpu > $O/pytest_b.log 2>&1 || { echo "pytest B failed"; tail -30 $O/pytest_b.log; exit 1; }
tail -1 $O/pytest_b.log
for v in A B; do
  E=""; [ $v = B ] && E="$AB"
  env SVTGPU_SR_STATS=1 $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing > $O/stats_$v.log 2>&1 || { echo "stats $v failed"; tail -20 $O/stats_$v.log; exit 1; }
  echo "$v $(grep sgr_res $O/stats_$v.log | tail -1)"
done
for f in 1 4; do
  for v in A B; do
    E=""; [ $v = B ] && E="$AB"
    env $E timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight $f > $O/b_${v}_f$f.log 2>&1 || { echo "bench $v failed"; tail -20 $O/b_${v}_f$f.log; exit 1; }
    echo "$v F=$f $(grep '^{' $O/b_${v}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]; print(d["value"], c["frame_latency_ms"], c["lr_search_kernel_ms"], r["kernel"], r["avg_launch_ms"])')"
  done
done
echo done
