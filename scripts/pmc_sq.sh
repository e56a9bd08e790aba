#!/bin/bash
# SQ counters of the main kernels at one frame in flight, two passes (<= 8 SQ counters each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K="sgr_flt|sgr_mom|cdef_search|cdef_apply|md_dist|lr_apply|dlf_tile|wiener_unit|sgr_queue|wiener_stats"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --frames-in-flight 1 --no-kernel-timing"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "$K" -d gpurun_out/pmcA -o run --output-format csv -- $B > gpurun_out/pmcA.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC --kernel-include-regex "$K" -d gpurun_out/pmcB -o run --output-format csv -- $B > gpurun_out/pmcB.log 2>&1
echo "exit $?"
