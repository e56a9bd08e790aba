set -o pipefail
# SQ counters of the LR search kernels (one frame in flight): VALU instructions, wave cycles and waits per kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "wiener_trial|proj_err|sgr_flt|sgr_mom|wiener_stats|cdef_search|dlf_tile|sod_step" -d gpurun_out/pmc1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --frames-in-flight 1 --no-kernel-timing > gpurun_out/pmc1.log 2>&1
echo "exit $?"
