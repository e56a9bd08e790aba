#!/bin/bash
# LR / pipeline GPU tests (incl. the row-part and tree variants), the self-guided search statistics (SVTGPU_SR_STATS) and
# the bench at F = 1 / 3 into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-src}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -k "lr or sgr or pipeline or rtcd" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
SVTGPU_SR_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix --frames-in-flight 1 --no-kernel-timing > $O/stats.log 2>&1 || { echo "stats failed"; tail -5 $O/stats.log; exit 1; }
grep sgr_res $O/stats.log | tail -1
for f in 1 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight $f > $O/b_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/b_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["stage_ms"]["lr_search_apply"], c["lr_search_kernel_ms"])')"
done
