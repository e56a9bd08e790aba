#!/bin/bash
# Round-6 profile of the default bench build (the figures bench.py's roofline reads back):
#   1. FETCH_SIZE / WRITE_SIZE calibration (scripts/ubench/fetch_cal.hip: known 1 GiB reads / writes);
#   2. FETCH_SIZE and WRITE_SIZE passes over the bench (separate: they do not fit one TCC pass);
#   3. two SQ passes (<= 8 SQ counters each): VALU / LDS instructions, wave cycles and waits, LDS bank conflicts;
#   4. rocprofv3 --kernel-trace --stats of the bench at one frame in flight and at the default four.
# As in round 5, the F = 1 passes run with --lr-serial (the LR chains one after the other, the condition of the bench
# line's isolated roofline phase), so the trace reproduces the line's launch durations.
# Each step under its own time limit; the script stops at the first failure.  Output under gpurun_out/r06prof.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${PROF_OUT:-r06prof}
mkdir -p $O
export TMPDIR=/tmp
K="lr_fin|lr_records|dlf_trial_dev|dlf_finish|md_expand|sgr_best|pick_final|pick_settle|wiener_res|sgr_res|sgr_flt|sgr_sse|unit_sums|wiener_stats|wiener_solve|cdef_search|cdef_apply|sod_step|dlf_tile|dlf_edge|lr_apply|md_dist"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --no-kernel-timing --lr-serial"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/ubench/fetch_cal.hip -o $O/fetch_cal &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal_fetch -o run --output-format csv -- $O/fetch_cal > $O/cal.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cal_write -o run --output-format csv -- $O/fetch_cal >> $O/cal.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/bench_fetch -o run --output-format csv -- $B > $O/bench_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/bench_write -o run --output-format csv -- $B > $O/bench_write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "$K" -d $O/sqA -o run --output-format csv -- $B > $O/sqA.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "$K" -d $O/sqB -o run --output-format csv -- $B > $O/sqB.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_f1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection --frames-in-flight 1 --lr-serial > $O/trace_f1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_f4 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-matrix --no-tile-projection > $O/trace_f4.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
