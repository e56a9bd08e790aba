#!/bin/bash
# Kernel-trace profiles (F=3, F=1) and the PMC traffic passes of the current build, without the test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-matrix > gpurun_out/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-matrix --frames-in-flight 1 > gpurun_out/prof1.log 2>&1 || exit $?
bash scripts/pmc_traffic.sh
