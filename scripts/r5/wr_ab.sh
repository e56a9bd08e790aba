#!/bin/bash
# Wiener descent A/B of two builds (in-tree vs $LIB): parity tests, SVTGPU_WR_STATS at one frame in flight, then the
# bench at F = 1 / 4 (the roofline's isolated phase times each LR kernel alone), alternating twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5wrab}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_lr_gpu.py tests/test_pipeline_golden.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5"
for rep in 1 2; do
  for L in svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so $LIB; do
    t=$(basename $L .so)
    SVTGPU_LIB=$L SVTGPU_WR_STATS=1 timeout -k 10 300 $B --frames-in-flight 1 > $O/${t}_stats_$rep.log 2>&1 || { echo "$t stats failed"; exit 1; }
    echo "$t stats: $(grep 'wiener_res:' $O/${t}_stats_$rep.log | tail -1)"
    SVTGPU_LIB=$L timeout -k 10 300 $B --frames-in-flight 4 > $O/${t}_f4_$rep.log 2>&1 || { echo "$t F=4 failed"; exit 1; }
    echo "$t F=4: $(grep '^{' $O/${t}_f4_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["all_kernels_ms_per_frame"])')"
  done
done
