#!/bin/bash
# A/B of an environment switch ($AB applied to B) on parity and on throughput at one and four frames in flight, plus
# the emulated largest rank of an 8-GPU tiled picture (bench.py --emulate-rank 8), into gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4ab2}
mkdir -p $O
T="python -u -m pytest -x -q --timeout 250 --timeout-method thread"
timeout -k 10 700 $T tests/test_cdef_gpu.py tests/test_dlf_gpu.py tests/test_dlf_device_gpu.py tests/test_pipeline_golden.py tests/test_lr_gpu.py tests/test_tiled_gpu.py -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for run in "1 0" "4 0" "4 8"; do
  set -- $run
  for v in A B; do
    E=""; [ $v = B ] && E="$AB"
    X=""; [ $2 -gt 0 ] && X="--emulate-rank $2"
    env $E timeout -k 10 300 python bench.py --steps 40 --warmup 4 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight $1 $X --host-timing > $O/b_${v}_f$1_e$2.log 2>&1 || { echo "bench $v $run failed"; tail -20 $O/b_${v}_f$1_e$2.log; exit 1; }
    echo "$v F=$1 emu=$2 $(grep '^{' $O/b_${v}_f$1_e$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; h=c.get("host_ms",{}); print(d["value"], c["frame_latency_ms"], c["stage_ms"]["dlf_pick_filter"], c["stage_ms"]["cdef_pick_apply"], c["stage_ms"]["lr_search_apply"], {k: h[k][0] for k in ("dlf_pick","cdef_pick","lr_search") if k in h})')"
  done
done
echo done
