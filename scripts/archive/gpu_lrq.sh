#!/bin/bash
# LR parity (queue kernel) then F=1 and F=3 benches; each GPU step time-limited, first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-lrq}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "lr or pipeline or rtcd" > $OUT/pytest.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --frames-in-flight 1 > $OUT/bench_f1.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_f3.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
echo "exit $rc"
exit $rc
