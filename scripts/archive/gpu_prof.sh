#!/bin/bash
# Kernel-trace profile of the default bench (rocprofv3 --kernel-trace --stats, csv) into gpurun_out/$1, plus a
# 2-rank gloo rehearsal of `--gpus 2` (bench.py spawns its own ranks) on the one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rp -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 2 --split frames --dist-backend gloo --steps 5 --warmup 1 --no-cpu-baseline > $OUT/gloo2_frames.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
