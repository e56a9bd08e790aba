#!/bin/bash
# Resident self-guided search diagnostics (SVTGPU_SR_STATS): per-item passes, candidates and load / descent / control
# times for each tree size at one frame in flight, then the default bench per tree size at F = 1 / 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/srstats
mkdir -p $O
export TMPDIR=/tmp
for t in 7 3 1; do
  SVTGPU_SR_STATS=1 SVTGPU_SR_TREE=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matrix \
      --frames-in-flight 1 --no-kernel-timing > $O/stats_t$t.log 2>&1 || { echo "stats run failed"; tail -20 $O/stats_t$t.log; exit 1; }
  echo "tree $t: $(grep sgr_res $O/stats_t$t.log | tail -1)"
done
for t in 7 3 1; do
  for f in 1 3; do
    SVTGPU_SR_TREE=$t timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix \
        --frames-in-flight $f > $O/b_t${t}_f$f.log 2>&1 || { echo "bench failed"; tail -20 $O/b_t${t}_f$f.log; exit 1; }
    echo "tree $t F=$f $(grep '^{' $O/b_t${t}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["frame_latency_ms"], c["stage_ms"]["lr_search_apply"], c["lr_search_kernel_ms"])')"
  done
done
