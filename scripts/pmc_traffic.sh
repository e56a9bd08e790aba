#!/bin/bash
# HBM-side traffic per launch for bench.py's roofline: FETCH_SIZE and WRITE_SIZE in separate passes (they do not
# fit one TCC pass), plus the fetch_cal calibration of both counters for the access widths the kernels use.
# Output: gpurun_out/traffic/{cal_fetch,cal_write,bench_fetch,bench_write}/..._counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/traffic
export TMPDIR=/tmp
K="sgr_flt|sgr_mom|wiener_unit|sgr_queue|wiener_stats|cdef_search|cdef_apply|dlf_tile|lr_apply|md_dist|unit_sums"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/ubench/fetch_cal.hip -o gpurun_out/traffic/fetch_cal &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/traffic/cal_fetch -o run --output-format csv -- gpurun_out/traffic/fetch_cal > gpurun_out/traffic/cal.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/traffic/cal_write -o run --output-format csv -- gpurun_out/traffic/fetch_cal >> gpurun_out/traffic/cal.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d gpurun_out/traffic/bench_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix > gpurun_out/traffic/bench_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d gpurun_out/traffic/bench_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix > gpurun_out/traffic/bench_write.log 2>&1
echo "exit $?"
