#!/bin/bash
# Bench variants in one call: BENCH_ARGS = ';'-separated argument sets, each optionally starting with
# "VAR=value ..." environment assignments; then an optional 2-rank gloo rehearsal (GLOO_ARGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra V <<< "$BENCH_ARGS"
for v in "${V[@]}"; do
  echo "== $v" >> gpurun_out/sweep.log
  envs=(); args=()
  for w in $v; do if [[ "$w" == *=* && "$w" != --* ]]; then envs+=("$w"); else args+=("$w"); fi; done
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline "${args[@]}" >> gpurun_out/sweep.log 2>&1 || exit 1
done
if [ -n "$GLOO_ARGS" ]; then
  echo "== gloo2 $GLOO_ARGS" >> gpurun_out/sweep.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline $GLOO_ARGS >> gpurun_out/sweep.log 2>&1 || exit 1
fi
echo "exit 0"
