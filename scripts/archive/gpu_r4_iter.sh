#!/bin/bash
# Round-4 iteration: LR parity tests, then the resident self-guided search diagnostics and the bench at F = 1 / 4,
# into gpurun_out/$1.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4iter}
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 250 --timeout-method thread"
timeout -k 10 600 $T tests/test_lr_gpu.py tests/test_pipeline_golden.py tests/test_lr_modes_gpu.py tests/test_tiled_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SVTGPU_WR_STATS=1 SVTGPU_SR_STATS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing > $O/stats.log 2>&1 || { echo "stats failed"; tail -20 $O/stats.log; exit 1; }
grep -E "sgr_res|wiener_res" $O/stats.log | tail -2
for f in 1 4; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight $f > $O/b_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_f$f.log; exit 1; }
  echo "F=$f $(grep '^{' $O/b_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"], c["lr_search_kernel_ms"], r["kernel"], r["avg_launch_ms"])')"
done
if [ -n "$PROJ" ]; then
  timeout -k 10 400 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix > $O/b_proj.log 2>&1 || { echo "projection bench failed"; tail -20 $O/b_proj.log; exit 1; }
  grep '^{' $O/b_proj.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["config"]["tile_projection"]; print(d["value"], {k: (v["projected_Mpx_s"], v["ms_per_step"], v["cdef_pick_ms"]) for k, v in p.items() if k != "note"})'
fi
echo done
