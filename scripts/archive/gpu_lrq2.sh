#!/bin/bash
# LR/pipeline parity with the Wiener queue, then F=1 benches over worker counts and the per-round path, then F=3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-lrq}
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "lr or pipeline or rtcd" > $OUT/pytest.log 2>&1 &&
SVTGPU_WN_QGRID=256 timeout -k 10 200 $B --frames-in-flight 1 > $OUT/f1_q256.log 2>&1 &&
SVTGPU_WN_QGRID=512 timeout -k 10 200 $B --frames-in-flight 1 > $OUT/f1_q512.log 2>&1 &&
SVTGPU_WN_QGRID=1024 timeout -k 10 200 $B --frames-in-flight 1 > $OUT/f1_q1024.log 2>&1 &&
SVTGPU_WN_QUEUE=0 timeout -k 10 200 $B --frames-in-flight 1 > $OUT/f1_rounds.log 2>&1 &&
SVTGPU_WN_QGRID=512 timeout -k 10 200 $B > $OUT/f3_q512.log 2>&1 &&
SVTGPU_WN_QUEUE=0 timeout -k 10 200 $B > $OUT/f3_rounds.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
echo "exit $rc"
exit $rc
