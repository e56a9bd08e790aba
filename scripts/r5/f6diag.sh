#!/bin/bash
# F = 6 diagnostics: the whole-frame bench at six frames in flight (default queues, then 20 queues), and the emulated
# rank of an 8-GPU tiled picture (its default: six frames in flight).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5f6}
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-matrix --no-tile-projection --steps 30 --warmup 5"
s() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c.get("frame_latency_ms"), {k: round(v, 2) for k, v in c["stage_ms"].items() if k != "note"})'; }
timeout -k 10 300 $B --frames-in-flight 6 > $O/f6.log 2>&1 || { echo "f6 failed"; tail $O/f6.log; exit 1; }; echo "F=6: $(s $O/f6.log)"
SVTGPU_BENCH_QUEUES=20 timeout -k 10 300 $B --frames-in-flight 6 > $O/f6q20.log 2>&1 || { echo "f6q20 failed"; exit 1; }; echo "F=6 q20: $(s $O/f6q20.log)"
timeout -k 10 300 $B --emulate-rank 8 > $O/e8.log 2>&1 || { echo "e8 failed"; tail $O/e8.log; exit 1; }; echo "emulated rank 8: $(s $O/e8.log)"
timeout -k 10 300 $B --frames-in-flight 4 > $O/f4.log 2>&1 || { echo "f4 failed"; exit 1; }; echo "F=4: $(s $O/f4.log)"
