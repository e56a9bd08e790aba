// svtgpu_internal.h — shared host/device definitions of the MI355X in-loop-filter library.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/svtgpu.h"

#define SVTGPU_VERSION_STR "svtgpu 0.1.0 (gfx950)"

// ---------------------------------------------------------------------------------------------
// error plumbing (never throws across the C ABI)
// ---------------------------------------------------------------------------------------------
#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            svtgpu_set_last_hip_error(e_, #expr, __FILE__, __LINE__);                         \
            return SVTGPU_ERR_HIP;                                                            \
        }                                                                                     \
    } while (0)

void svtgpu_set_last_hip_error(hipError_t e, const char *what, const char *file, int line);
// Per-block RTCD shims cannot return an error through their reference signature: abort loudly.
[[noreturn]] void svtgpu_fatal(const char *what);
#define HIP_OR_DIE(expr)                                                                      \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            svtgpu_set_last_hip_error(e_, #expr, __FILE__, __LINE__);                         \
            svtgpu_fatal(#expr);                                                              \
        }                                                                                     \
    } while (0)

// ---------------------------------------------------------------------------------------------
// objects
// ---------------------------------------------------------------------------------------------
struct SvtGpuContext {
    int         device;
    hipStream_t stream;
};

struct SvtGpuFrame {
    SvtGpuContext *ctx;
    int32_t        width, height, bit_depth;
    int32_t        bytes_per_sample;
    int32_t        pw[3], ph[3]; // plane sizes
    int32_t        stride[3];    // samples
    void          *plane[3];     // device pointers (one allocation)
    void          *base;
};

// frame geometry in 4x4 mode-info units (SB64 CDEF filter blocks of 16x16 mi)
struct FrameGeo {
    int32_t mi_rows, mi_cols, nvfb, nhfb, b8_rows, b8_cols;
};
static inline FrameGeo frame_geo(int32_t w, int32_t h) {
    FrameGeo g;
    g.mi_cols = ((w + 7) & ~7) >> 2;
    g.mi_rows = ((h + 7) & ~7) >> 2;
    g.nhfb    = (g.mi_cols + 15) / 16;
    g.nvfb    = (g.mi_rows + 15) / 16;
    g.b8_cols = g.mi_cols / 2;
    g.b8_rows = g.mi_rows / 2;
    return g;
}

// A high-priority lane for a call's latency-bound launch chains (the CDEF pick's 41 dependent steps, the DLF level
// search's trial launches): the work forks from the caller's stream onto a stream of the greatest priority and joins
// back, so stream order for the caller is unchanged, and the dispatcher hands those small launches the next free CU
// slots instead of queueing them behind other frames' resident kernels.  Opt-in (SVTGPU_HIPRIO=1): measured slower
// (runtime.hip).
struct SvtGpuPrioLane {
    hipStream_t hs   = nullptr;
    hipEvent_t  fork = nullptr, join = nullptr;
};
// the stream to launch on (the lane's, or `st` itself when the lane is off); svtgpu_prio_leave joins it back into st
int  svtgpu_prio_enter(SvtGpuPrioLane *l, hipStream_t st, hipStream_t *out);
int  svtgpu_prio_leave(SvtGpuPrioLane *l, hipStream_t hs, hipStream_t st);
void svtgpu_prio_destroy(SvtGpuPrioLane *l);

// persistent pick exchange (cdef_pick.hip): [64 chunks][4 chains][4096] partial sums, [4][64][2] row minima,
// then status and diagnostics words
#define SVTGPU_PICK_XCH_BYTES ((size_t)(64 * 4 * 4096 + 4 * 64 * 2 + 16) * 8)

struct SvtGpuCdefFrameState {
    SvtGpuContext *ctx;
    int32_t        width, height;
    FrameGeo       geo;
    int32_t        nfb;
    uint8_t       *d_mask;        // [b8_rows][b8_cols] 1 = filter block
    uint64_t      *d_mse;         // [2][nfb][64]
    uint8_t       *d_skip;        // [nfb]
    uint8_t       *d_dir;         // [nfb][64]
    int32_t       *d_var;         // [nfb][64]
    int8_t        *d_fb_strength; // [nfb]
    // pick scratch
    uint64_t      *d_pick_part;   // partial tot_mse tables
    uint64_t      *d_pick_out;    // [chains][4] (best, j, k)
    int32_t       *d_pick_lev;    // [chains][2][16]
    int32_t       *d_fb_list;     // compacted non-skip FB indices [nfb], their count, FB -> index or -1 [nfb]
    uint64_t      *d_pick_xch;    // persistent pick: tagged partial sums, row minima, status, diagnostics (cdef_pick.hip)
    uint32_t       pick_epoch;    // picks run by the persistent kernel (tags its exchange words)
    int32_t        pick_settle;   // the launch path's settle checkpoint: the step after which the pick checks
    int32_t        pick_miss;     // consecutive checks that found a chain unsettled
    int32_t        pick_skip;     // picks left that run without the check (after 2 misses: 8)
    int32_t        pick_xch_end;  // the strength count of the words in d_pick_xch (0: none written)
    uint8_t       *h_pick;        // pinned, mapped: the pick's result (PickOut) then the per-FB strengths [nfb]
    uint8_t       *h_pick_dev;    // its device address
    int32_t        pick_parts;
    int32_t        mask_all;      // mask == every block
    int32_t        fb_rect[4];    // {col0, row0, col1, row1}: the filter blocks searched (tiling over GPUs)
    int32_t        out_rect[4];   // {x0, y0, x1, y1} luma: the samples the apply writes (tiling over GPUs)
    SvtGpuComm    *comm;          // the pick's exchange of the search tables (tiling over GPUs; null: none)
    int32_t        gathered;      // the tables already hold every rank's blocks (summed since the last search)
    uint64_t      *own_mse;       // state-owned tables (d_mse/d_skip may point at caller memory)
    uint8_t       *own_skip;      // [nfb rounded up to 8]: the padding stays 0 (the skip table's word sums)
    uint8_t       *own_dir;       // state-owned dir/var (d_dir/d_var may point at caller memory)
    int32_t       *own_var;
    int8_t        *d_fb_kind;     // [nfb] SB128 areas (cdef_sb128.hip); null = SB64
    int8_t        *h_fb_kind;     // host copy
    uint8_t       *d_mse_rem;     // [3][nfb][64] remainders of the per-FB distortion shift (SB128 only)
    SvtGpuPrioLane prio;          // the pick's launch chain
    // svtgpu_cdef_pick_async: [0] the settle check's flag for the later steps, [16..] the parameters the apply reads
    void          *d_apick;
    int32_t        settle_seq, settle_seen; // settle checks enqueued / the last one whose record the host has taken
    int32_t        apick_seq;               // asynchronous picks enqueued (the record's seq)
    int32_t        apick_pending, apick_ready, apick_ref; // a result not yet read; device parameters exist; ref-fs
    SvtGpuCdefParams apick_params;          // ref-fs: the parameters (known at enqueue)
    uint8_t        apick_map[64], apick_damping; // the strength map of the pending pick (its read-back)
};

// Device-side view of the searched strengths (built on the host from SvtGpuCdefControls).
// The CDEF tap sum splits into a primary part that depends only on the primary strength and a
// secondary part that depends only on the secondary strength (EbCdef.c:263-297), so strengths are
// grouped by (tap direction set, primary level) and the secondary sums are shared.
struct CdefGroupTable {  // strengths evaluated with one tap-direction set
    int32_t nlv;         // number of primary levels in the group
    int32_t sec_used;    // bitmask of secondary codes (1..3) used by the group
    int32_t lv[16];      // primary levels
    int32_t gi[16][4];   // gi of (level idx, secondary code) or -1
};
struct CdefStrengthTable {
    int32_t        nstr;      // total strengths searched (first + second pass)
    CdefGroupTable luma[2];   // [0]: primary level 0 (direction-0 taps), [1]: block direction
    CdefGroupTable chroma[2]; // same, chroma-tested strengths only
    uint8_t        uv_on[64]; // gi -> chroma tested
    int8_t         alias[64]; // gi -> earlier gi with the same strength code (or -1)
};

// ---------------------------------------------------------------------------------------------
// launchers (defined in the .hip translation units)
// ---------------------------------------------------------------------------------------------
int svtgpu_launch_cdef_search(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, const SvtGpuFrame *src,
                              const CdefStrengthTable *tab, int32_t subsampling, int32_t damping,
                              hipStream_t st);
int  svtgpu_launch_cdef_sb128_fold(SvtGpuCdefFrameState *s, unsigned long long uv_on, int cs, int ss, hipStream_t st);
int  svtgpu_launch_cdef_sb128_dup(SvtGpuCdefFrameState *s, hipStream_t st);
void svtgpu_cdef_sb128_dup_host(const SvtGpuCdefFrameState *s, int8_t *fbs);
// p == nullptr: the parameters the last asynchronous pick left in device memory
int svtgpu_launch_cdef_apply(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, SvtGpuFrame *out,
                             const SvtGpuCdefParams *p, hipStream_t st);
// the asynchronous pick's device parameters set to `p` in stream order (the reference-fs case: no search)
int svtgpu_launch_cdef_set_params(SvtGpuCdefFrameState *s, const SvtGpuCdefParams *p, hipStream_t st);

// the default context's stream (per-block shims and stream-less frame-level calls)
hipStream_t svtgpu_default_stream();
// the same stream, counted as one per-block shim call (svtgpu_shim_calls): used once per RTCD shim entry point only
hipStream_t svtgpu_shim_stream();
// svt_av1_compute_stats(_highbd) of one unit on the matrix cores (lr_search.hip; 8- and 10-bit samples)
int svtgpu_stats_unit_mfma8(int win, const uint8_t *dgd, const uint8_t *src, int h_start, int h_end, int v_start,
                            int v_end, int dgd_stride, int src_stride, int64_t *M, int64_t *H);
int svtgpu_stats_unit_mfma16(int win, const uint16_t *dgd, const uint16_t *src, int h_start, int h_end, int v_start,
                             int v_end, int dgd_stride, int src_stride, int64_t *M, int64_t *H, int div);
// Host wait for a small device result: the kernel's last workgroup writes the payload into mapped pinned memory,
// then (after a system-scope fence) the sequence word `seq`.  Spinning on that word returns as soon as it lands;
// the stream's own synchronize wakes the host up tens of microseconds later, once per host round trip.  Falls
// back to synchronizing `st` (and fails if the word is still missing after it).
int svtgpu_wait_seq(const volatile unsigned long long *flag, unsigned long long seq, hipStream_t st);
// element-wise sum of n uint64 over the ranks of `c` (comm.hip); nullptr or a one-rank comm: nothing to do.  `what`
// names the exchange in a timeout's message (SVTGPU_XCH_*)
int svtgpu_comm_sum(SvtGpuComm *c, void *buf, size_t n, bool on_device, hipStream_t st, const char *what);
#define SVTGPU_XCH_DLF "DLF trial SSEs"
#define SVTGPU_XCH_CDEF "CDEF search tables"
#define SVTGPU_XCH_LR "LR search records"
// host wait for `st`, bounded by c's deadline while one of its device-side collectives is outstanding (comm.hip);
// c == nullptr: hipStreamSynchronize
int svtgpu_comm_wait(SvtGpuComm *c, hipStream_t st);
// the tiled (gather) path runs: a comm of several ranks, or a one-rank RCCL comm (the N-GPU code path on one device)
bool svtgpu_comm_tiled(const SvtGpuComm *c);
// host <-> device bytes of the frame-level entry points (copies and mapped-memory results), for the bench's report
void svtgpu_count_xfer(int d2h, size_t bytes);
SvtGpuContext *svtgpu_default_context();
static inline hipStream_t pick_stream(SvtGpuContext *ctx, void *stream) {
    return stream ? (hipStream_t)stream : ctx->stream;
}

// Diagnostics (SVTGPU_WGCLK=<file>, never on by default): per workgroup 8 words -- up to 6 time marks on the 100 MHz
// s_memrealtime clock (slot 0 = start; the kernel's phases after it; unused slots stay 0) and the hardware id words
// (HW_ID: wave / SIMD / CU / SE; XCC_ID) -- appended to the file by the launching host code (svtgpu_wgclk_*).
// Written by lane 0 with vector stores.
__device__ __forceinline__ void wgclk_mark(unsigned long long *buf, int slot) {
    if (!buf || threadIdx.x) return;
    unsigned long long *q = buf + 8 * (size_t)blockIdx.x;
    q[slot]               = __builtin_amdgcn_s_memrealtime();
    if (!slot) {
        q[6] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4); // HW_REG_HW_ID
        q[7] = (unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20); // HW_REG_XCC_ID
    }
}
unsigned long long *svtgpu_wgclk_begin(int nblocks);               // null unless SVTGPU_WGCLK is set
void                svtgpu_wgclk_end(const char *kernel, int nblocks, hipStream_t st); // sync + append

// XCD-aware block order (speed only, never correctness): workgroups are dealt round-robin over the 8 XCDs, so
// blocks b, b + 8, ... share one XCD's L2.  Give each such group a contiguous range of logical indices so tiles that
// share halo lines (the neighbours of a row-major tile list) are read through the same L2.  Bijective for any n.
__device__ __forceinline__ int xcd_swizzle(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// ---------------------------------------------------------------------------------------------
// Wave64 reductions with DPP (VALU only; no ds_bpermute chains): row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast 15 / 31 across rows.  The total lands in lane 63 (the other lanes hold partial sums).
// ---------------------------------------------------------------------------------------------
template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROW_MASK, BANK_MASK, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROW_MASK, BANK_MASK, true);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ unsigned long long wave_sum_lane63(unsigned long long v) {
    v += dpp_u64<0x111, 0xf, 0xf>(v); // row_shr:1
    v += dpp_u64<0x112, 0xf, 0xf>(v); // row_shr:2
    v += dpp_u64<0x114, 0xf, 0xe>(v); // row_shr:4, banks 1-3
    v += dpp_u64<0x118, 0xf, 0xc>(v); // row_shr:8, banks 2-3
    v += dpp_u64<0x142, 0xa, 0xf>(v); // row_bcast:15 into rows 1 and 3
    v += dpp_u64<0x143, 0xc, 0xf>(v); // row_bcast:31 into rows 2 and 3
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32_lane63(uint32_t v) { // 32-bit DPP adds (mod 2^32)
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xe, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xc, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, true);
    return v;
}
// exact 64-bit wave total (lane 63) of per-lane u32 values: two 16-bit limbs (each limb sum < 2^22)
__device__ __forceinline__ unsigned long long wave_sum_u32_wide(uint32_t v) {
    return (unsigned long long)wave_sum_u32_lane63(v & 0xFFFFu) +
           ((unsigned long long)wave_sum_u32_lane63(v >> 16) << 16);
}
// exact wave total (lane 63) of per-lane int32 values, as int64
__device__ __forceinline__ long long wave_sum_i32_wide(int v) {
    return (long long)wave_sum_u32_wide((uint32_t)v ^ 0x80000000u) - 64ll * 0x80000000ll;
}
// exact wave total (lane 63) of per-lane 64-bit values mod 2^64: three 22-bit limbs (each limb sum < 2^28)
__device__ __forceinline__ unsigned long long wave_sum_u64_limbs(unsigned long long v) {
    const uint32_t l0 = (uint32_t)(v & 0x3FFFFF), l1 = (uint32_t)((v >> 22) & 0x3FFFFF), l2 = (uint32_t)(v >> 44);
    return (unsigned long long)wave_sum_u32_lane63(l0) + ((unsigned long long)wave_sum_u32_lane63(l1) << 22) +
           ((unsigned long long)wave_sum_u32_lane63(l2) << 44);
}
