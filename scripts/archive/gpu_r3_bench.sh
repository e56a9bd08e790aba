#!/bin/bash
# Round-3 bench checks: N=1 at one and three frames in flight, then the N=2 tiled path rehearsed with two ranks on
# the one GPU (host transport over gloo) and the frames split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bench
export TMPDIR=/tmp
summ() { grep '^{' "$1" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]; print(d["value"], d["scaling"], c["parallelism"][:30], c["frame_latency_ms"], c["stage_ms"], r["kernel"], r["frac"], r["ms_per_frame"])'; }
for f in 1 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-matrix --frames-in-flight $f > gpurun_out/bench/n1_f$f.log 2>&1 || { tail -20 gpurun_out/bench/n1_f$f.log; exit 1; }
  echo "N=1 F=$f $(summ gpurun_out/bench/n1_f$f.log)"
done
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-matrix --master-port 29611 > gpurun_out/bench/n2_tiles_gloo.log 2>&1 || { tail -30 gpurun_out/bench/n2_tiles_gloo.log; exit 1; }
echo "N=2 tiles(gloo, 1 GPU) $(summ gpurun_out/bench/n2_tiles_gloo.log)"
timeout -k 10 400 python bench.py --gpus 2 --split frames --steps 10 --warmup 2 --no-matrix --master-port 29612 > gpurun_out/bench/n2_frames.log 2>&1 || { tail -30 gpurun_out/bench/n2_frames.log; exit 1; }
echo "N=2 frames(1 GPU) $(summ gpurun_out/bench/n2_frames.log)"
