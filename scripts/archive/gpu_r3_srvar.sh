#!/bin/bash
# Resident self-guided search variants: the default build (1024-lane workgroups) and scripts/ubench/var/
# libsvtgpu_sr512.so (512-lane workgroups, two per CU), trees of 1 and 3 nodes: pipeline goldens (variant), per-item
# diagnostics (SVTGPU_SR_STATS) and the bench at F = 1 / 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/srvar
mkdir -p $O
export TMPDIR=/tmp
LIB=svt-av1_pro-anchor-v2.1.0-_amd/lib/libsvtgpu.so
cp $LIB $O/lib_default.so
for v in default sr512; do
  if [ $v = sr512 ]; then cp scripts/ubench/var/libsvtgpu_sr512.so $LIB; fi
  timeout -k 10 600 python -u -m pytest tests/test_pipeline_golden.py tests/test_lr_modes_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; cp $O/lib_default.so $LIB; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  for t in 1 3; do
    SVTGPU_SR_STATS=1 SVTGPU_SR_TREE=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix \
        --frames-in-flight 1 --no-kernel-timing > $O/stats_${v}_t$t.log 2>&1 || { echo "stats failed"; tail -20 $O/stats_${v}_t$t.log; exit 1; }
    echo "$v tree $t: $(grep sgr_res $O/stats_${v}_t$t.log | tail -1)"
    for f in 1 3; do
      SVTGPU_SR_TREE=$t timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix \
          --frames-in-flight $f > $O/b_${v}_t${t}_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_${v}_t${t}_f$f.log; exit 1; }
      echo "$v tree $t F=$f $(grep '^{' $O/b_${v}_t${t}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"]["lr_search_apply"], c["lr_search_kernel_ms"])')"
    done
  done
done
cp $O/lib_default.so $LIB
