// dlf.hip — AV1 deblocking loop filter on gfx950: frame apply and full-image level search.
//
// Reference path (GabrielGao0310/SVT-av1_pro-anchor-v2.1.0-, Source/Lib/):
//   edge filters       Common/Codec/EbDeblockingCommon.c:141-373, 436-865 (lpf 4/6/8/14, 8-bit + highbd)
//   edge parameters    Encoder/Codec/EbDeblockingFilter.c:143-282 (get_transform_size, set_lpf_parameters)
//   level tables       Common/Codec/EbDeblockingCommon.c:76-139, 554-572; EbDeblockingFilter.c:35-47
//   frame passes       Encoder/Codec/EbDeblockingFilter.c:287-653 (SB-lagged vert/horz, combine_vert_horz_lf)
//   level search       Encoder/Codec/EbDeblockingFilter.c:716-991, 1129-1252 (FULL_IMAGE bisection)
//
// Design (MI355X):
//  * The mode-info grid is uploaded once per frame and turned into per-4x4 *edge records* per plane
//    type and direction: the filter length the transform/prediction geometry allows (0/4/6/8/14) and
//    the (segment, ref, mode) level classes of the two sides.  Everything that does not depend on
//    the filter level is resolved once; a level trial then only looks a level up in a 128-entry table.
//  * Within one direction no two edge segments touch the same samples (4-tap: p1..q1, 8-tap needs
//    8-wide transforms on both sides, 14-tap 16-wide), so the reference's SB-lagged order equals
//    "all vertical edges, then all horizontal edges" (the AV1 normative order).
//  * One workgroup per 64x64 tile: the tile plus a 12-sample apron is staged in LDS, the vertical
//    edges that reach the tile are filtered over the tile's rows and the apron rows, then the
//    horizontal edges over the tile's columns; the tile is either written out (apply) or compared with
//    the source for the SSE of a level trial — recon is never modified by a trial, so the search
//    needs no backup/restore copies, and a trial reads each sample once.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "svtgpu_internal.h"

#ifndef DLF_EXP
#define DLF_EXP 0 // development experiments (bit 0: no vertical pass, bit 1: no horizontal pass); 0 = real kernel
#endif

namespace {

// ---------------------------------------------------------------------------------------------
// AV1 size tables (BlockSize / TxSize enum order of EbDefinitions.h)
// ---------------------------------------------------------------------------------------------
constexpr int kNumBsize = 22;
// log2 of the transform width/height of tx_depth_to_tx_size[depth][bsize] (EbDefinitions.h:885-906)
__constant__ uint8_t c_tx_lw[3][kNumBsize] = {
    {2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 6, 2, 4, 3, 5, 4, 6},
    {2, 2, 3, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 2, 3, 3, 4, 4, 5},
    {2, 2, 3, 3, 2, 2, 2, 3, 3, 3, 4, 4, 4, 6, 6, 6, 2, 2, 3, 3, 4, 4}};
__constant__ uint8_t c_tx_lh[3][kNumBsize] = {
    {2, 3, 2, 3, 4, 3, 4, 5, 4, 5, 6, 5, 6, 6, 6, 6, 4, 2, 5, 3, 6, 4},
    {2, 3, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 3, 2, 4, 3, 5, 4},
    {2, 3, 2, 3, 2, 2, 2, 3, 3, 3, 4, 4, 4, 6, 6, 6, 2, 2, 3, 3, 4, 4}};
// 4:2:0 chroma: av1_get_max_uv_txsize (EbUtility.h:117-123, 64 -> 32) and the plane block size
// ss_size_lookup[bsize][1][1] (EbUtility.h:86-110), as log2 width / height
__constant__ uint8_t c_uvtx_lw[kNumBsize] = {2, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 5, 5, 2, 3, 2, 4, 3, 5};
__constant__ uint8_t c_uvtx_lh[kNumBsize] = {2, 2, 2, 2, 3, 2, 3, 4, 3, 4, 5, 4, 5, 5, 5, 5, 3, 2, 4, 2, 5, 3};
__constant__ uint8_t c_bs_lw[kNumBsize]   = {2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 7, 7, 2, 4, 3, 5, 4, 6};
__constant__ uint8_t c_bs_lh[kNumBsize]   = {2, 3, 2, 3, 4, 3, 4, 5, 4, 5, 6, 5, 6, 7, 6, 7, 4, 2, 5, 3, 6, 4};
__constant__ uint8_t c_uvbs_lw[kNumBsize] = {2, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 2, 3, 2, 4, 3, 5};
__constant__ uint8_t c_uvbs_lh[kNumBsize] = {2, 2, 2, 2, 3, 2, 3, 4, 3, 4, 5, 4, 5, 6, 5, 6, 3, 2, 4, 2, 5, 3};
// mode_lf_lut (EbDeblockingCommon.h:62-66): GLOBALMV (15) and GLOBAL_GLOBALMV (23) map to 0
__device__ __forceinline__ int mode_lf(int mode) { return mode >= 13 && mode != 15 && mode != 23; }

// Edge record (one per 4x4 unit per plane type and direction):
//   bits 0..3  filter length allowed by geometry (0, 4, 6, 8, 14)
//   bits 8..14 level class of the current block  (segment*16 + ref*2 + mode_lf)
//   bits 16..22 level class of the previous block
__device__ __forceinline__ int lf_class(const SvtGpuLfMi &m) {
    return m.segment_id * 16 + m.ref_frame0 * 2 + mode_lf(m.mode);
}

// log2 of the transform extent across the edge (get_transform_size + txsize_{horz,vert}_map)
__device__ __forceinline__ int tx_log2(const SvtGpuLfMi &m, int vert, int chroma) {
    const int skipped = m.skip && m.ref_frame0 > 0;
    if (chroma) return vert ? c_uvtx_lw[m.bsize] : c_uvtx_lh[m.bsize];
    const int d = skipped ? 0 : m.tx_depth;
    return vert ? c_tx_lw[d][m.bsize] : c_tx_lh[d][m.bsize];
}

// A record read from a grid that was not checked on the host (svtgpu_dlf_set_mode_info_device): fields outside the
// ranges the tables are indexed by raise *bad and are clamped, so no table read leaves its bounds.
__device__ __forceinline__ SvtGpuLfMi checked_mi(SvtGpuLfMi m, unsigned long long *bad) {
    if (bad && (m.bsize >= kNumBsize || m.tx_depth > 2 || m.ref_frame0 < 0 || m.ref_frame0 > 7 || m.mode > 24 ||
                m.segment_id > 7)) {
        *bad = 1;
        m.bsize = min((int)m.bsize, kNumBsize - 1), m.tx_depth = min((int)m.tx_depth, 2);
        m.ref_frame0 = (int8_t)min(max((int)m.ref_frame0, 0), 7), m.mode = min((int)m.mode, 24);
        m.segment_id = min((int)m.segment_id, 7);
    }
    return m;
}

__global__ void dlf_edge_records_kernel(const SvtGpuLfMi *__restrict__ mi, int mi_cols, int units_w, int units_h,
                                        int chroma, int vert, int crop_w, int crop_h, uint32_t *__restrict__ rec,
                                        unsigned long long *bad) {
    const int ux = blockIdx.x * blockDim.x + threadIdx.x;
    const int uy = blockIdx.y;
    if (ux >= units_w || uy >= units_h) return;
    const int ss     = chroma;
    const int x      = ux * 4, y = uy * 4;
    const int mi_row = ss | ((y << ss) >> 2), mi_col = ss | ((x << ss) >> 2);
    const SvtGpuLfMi m = checked_mi(mi[mi_row * mi_cols + mi_col], bad);
    const int coord    = vert ? x : y;
    uint32_t  r        = 0;
    const int lt       = tx_log2(m, vert, chroma);
    // an edge at or past the plane's unpadded size is not filtered (set_lpf_parameters, EbDeblockingFilter.c:173-178)
    if (coord && !(coord & ((1 << lt) - 1)) && x < crop_w && y < crop_h) { // a transform edge with a block beyond it
        const SvtGpuLfMi p = checked_mi(vert ? mi[mi_row * mi_cols + mi_col - (1 << ss)]
                                             : mi[(mi_row - (1 << ss)) * mi_cols + mi_col], bad);
        const int cur_skip = m.skip && m.ref_frame0 > 0;
        const int pv_skip  = p.skip && p.ref_frame0 > 0;
        const int lpb      = chroma ? (vert ? c_uvbs_lw[m.bsize] : c_uvbs_lh[m.bsize])
                                    : (vert ? c_bs_lw[m.bsize] : c_bs_lh[m.bsize]);
        const int pu_edge  = !(coord & ((1 << lpb) - 1));
        if (!pv_skip || !cur_skip || pu_edge) {
            const int mlt = min(lt, tx_log2(p, vert, chroma));
            const int len = mlt == 2 ? 4 : chroma ? 6 : mlt == 3 ? 8 : 14;
            r = (uint32_t)len | ((uint32_t)lf_class(m) << 8) | ((uint32_t)lf_class(p) << 16);
        }
    }
    rec[(size_t)uy * units_w + ux] = r;
}

// ---------------------------------------------------------------------------------------------
// one sample line across an edge: F[k] = sample at offset k-7 from the edge (p6 = F[0], q0 = F[7])
// AV1 narrow filter / wide filters (filter4/6/8/14 of EbDeblockingCommon.c)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int sclamp(int v, int lo, int hi) { return min(max(v, lo), hi); }

// wide filter with n taps per side (n = 2: 6-tap, 3: 8-tap, 6: 14-tap); outputs F[7-n .. 7+n-1]
template <int N, int LOG2>
__device__ __forceinline__ void wide_filter(int *F) {
    int out[2 * N];
#pragma unroll
    for (int i = -N; i < N; i++) {
        int t = 0;
#pragma unroll
        for (int j = -N; j <= N; j++) {
            const int p   = min(max(i + j, -(N + 1)), N);
            const int tap = (N == 3 ? j == 0 : (j >= -1 && j <= 1)) ? 2 : 1;
            t += F[p + 7] * tap;
        }
        out[i + N] = (t + (1 << (LOG2 - 1))) >> LOG2;
    }
#pragma unroll
    for (int i = -N; i < N; i++) F[i + 7] = out[i + N];
}

__device__ __forceinline__ void filter_line(int *F, int len, int blimit, int limit, int thresh, int bd) {
    const int sh = bd - 8, one = 1 << sh;
    const int p3 = F[3], p2 = F[4], p1 = F[5], p0 = F[6], q0 = F[7], q1 = F[8], q2 = F[9], q3 = F[10];
    const int lim = limit << sh;
    if (abs(p0 - q0) * 2 + abs(p1 - q1) / 2 > (blimit << sh)) return;
    int m = max(abs(p1 - p0), abs(q1 - q0));
    int flat = 0;
    if (len >= 6) {
        m = max(m, max(abs(p2 - p1), abs(q2 - q1)));
        flat = max(max(abs(p1 - p0), abs(q1 - q0)), max(abs(p2 - p0), abs(q2 - q0)));
    }
    if (len >= 8) {
        m    = max(m, max(abs(p3 - p2), abs(q3 - q2)));
        flat = max(flat, max(abs(p3 - p0), abs(q3 - q0)));
    }
    if (m > lim) return;
    if (len >= 6 && flat <= one) {
        if (len == 14) {
            const int flat2 = max(max(max(abs(F[2] - p0), abs(F[11] - q0)), max(abs(F[1] - p0), abs(F[12] - q0))),
                                  max(abs(F[0] - p0), abs(F[13] - q0)));
            if (flat2 <= one) {
                wide_filter<6, 4>(F);
                return;
            }
        }
        if (len == 6)
            wide_filter<2, 3>(F);
        else
            wide_filter<3, 3>(F);
        return;
    }
    // narrow filter (filter4)
    const int off = 0x80 << sh, lo = -(128 << sh), hi = (128 << sh) - 1;
    const bool hev = max(abs(p1 - p0), abs(q1 - q0)) > (thresh << sh);
    const int ps1 = p1 - off, ps0 = p0 - off, qs0 = q0 - off, qs1 = q1 - off;
    int f = hev ? sclamp(ps1 - qs1, lo, hi) : 0;
    f            = sclamp(f + 3 * (qs0 - ps0), lo, hi);
    const int f1 = sclamp(f + 4, lo, hi) >> 3;
    const int f2 = sclamp(f + 3, lo, hi) >> 3;
    F[7]         = sclamp(qs0 - f1, lo, hi) + off;
    F[6]         = sclamp(ps0 + f2, lo, hi) + off;
    if (!hev) {
        const int f3 = (f1 + 1) >> 1;
        F[8]         = sclamp(qs1 - f3, lo, hi) + off;
        F[5]         = sclamp(ps1 + f3, lo, hi) + off;
    }
}

__device__ __forceinline__ int half_taps(int len) { return len == 14 ? 7 : len == 8 ? 4 : len == 6 ? 3 : 2; }

// ---------------------------------------------------------------------------------------------
// tile kernel: apply (write) or level trial (SSE)
// ---------------------------------------------------------------------------------------------
constexpr int TILE  = 64;
constexpr int APRON = 12;
constexpr int LW    = TILE + 2 * APRON; // 88 samples per LDS row
constexpr int NTHR  = 256;
constexpr int MAX_TRIALS = 2; // levels per trial launch (the bisection's lo and hi candidates)

constexpr int MAX_JOBS   = 3; // planes per launch: the Y, U and V level searches run side by side

// one plane of a launch
struct DlfPlaneJob {
    int32_t         plane;    // 0 Y, 1 U, 2 V (the device level tables' index)
    const void     *src;      // recon plane (apply: a copy of it)
    void           *dst;      // apply output
    const void     *ref;      // source picture plane (trial)
    const uint32_t *rec_v, *rec_h; // edge records of this plane type
    int32_t         src_stride, dst_stride, ref_stride;
    int32_t         units_w;  // records per row (= pw / 4)
    int32_t         pw, ph, tiles_x, tiles;
    int32_t         ox, oy, ow, oh; // the region filtered / measured (a tile of a picture split over GPUs)
    int32_t         ntrial;
    uint8_t         lvl[MAX_TRIALS][2][128]; // [trial][dir][class] filter level
};

// a device-resident level search (svtgpu_dlf_pick with SVTGPU_DLF_DEVICE=1): the levels and level tables of the next
// trial launch, written by dlf_search_step_kernel from the previous launch's SSEs (no host decision between trials)
struct DlfDevPlan {
    int32_t ntrial[MAX_JOBS];                   // levels of each job in the next trial launch (0: the job has none)
    int32_t lv[MAX_JOBS][MAX_TRIALS];
    uint8_t lvl[MAX_JOBS][MAX_TRIALS][2][128];  // [job][trial][dir][class]
    int32_t done;                               // every search has finished
};

struct DlfTileArgs {
    DlfPlaneJob job[MAX_JOBS];
    int32_t     njob, bd;
    uint8_t     mblim[64], lim[64], hev[64];
    // trial mode: per-(job, trial) SSE accumulators and the count of finished workgroups, both zero between
    // launches (the last workgroup hands the sums to `out` -- mapped pinned host memory -- and re-zeroes them)
    unsigned long long *sse;
    unsigned int       *arrive;
    unsigned long long *out; // [MAX_JOBS][MAX_TRIALS] sums, then the sequence word (svtgpu_wait_seq)
    unsigned long long  seq;
    unsigned long long *wgclk; // diagnostics (svtgpu_internal.h wgclk_mark) or null
    const DlfDevPlan   *plan;  // trial mode: levels from the device plan (the grid covers MAX_TRIALS per job) or null
    DlfDevPlan         *next_plan = nullptr; // the asynchronous search: the plan buffer the next trial launch reads (or null)
    int32_t             dyn;   // with plan: the items are the plan's levels only, Σ tiles x plan->ntrial (persistent grid)
    const uint8_t      *dev_lvl; // apply: the level tables [plane][dir][128] the device search left (null: job lvl[0])
};

// The launch arguments as the kernels' items read them: in the kernarg segment (constant address space, scalar
// loads).  A reference to the by-value kernel parameter passed into the item function made the compiler copy the
// 2 KB argument block to scratch (private segment 2168 B, 13 VGPRs spilled); the kernarg pointer keeps it in place
// (the argument block is every launch's first parameter, at offset 0).
typedef const __attribute__((address_space(4))) DlfTileArgs KArgs;
typedef const __attribute__((address_space(4))) DlfPlaneJob KJob;
__device__ __forceinline__ KArgs &kargs() { return *(KArgs *)__builtin_amdgcn_kernarg_segment_ptr(); }

// the LDS of one tile item (dlf_tile_item); the persistent trial kernel's last workgroup reuses `t` for the step
struct DlfTileLds {
    uint16_t t[LW * LW];
    uint32_t rv[(LW / 4) * (TILE / 4 + 3)]; // vertical-edge records: 22 rows x 19 edges
    uint32_t rh[(TILE / 4 + 3) * (TILE / 4)]; // horizontal-edge records: 19 edges x 16 cols
    unsigned long long red[NTHR / 64];
    // this workgroup's level table (per direction and level class) and the per-level thresholds (mblim | lim << 8 |
    // hev << 16), looked up per edge with lane-varying indices: from LDS, not from the kernel arguments (a lane-varying
    // index into the argument block is a memory load per lookup)
    uint8_t  s_lvl[2][128];
    uint32_t s_thr[64];
    uint16_t s_list[(LW / 4) * (TILE / 4 + 3)]; // list_edges (>= the horizontal count, 19 x 16)
    int      s_cnt[8];
};

// The edges of one direction that filter anything (a length and a nonzero level on either side), listed in LDS
// grouped by filter length (4, 6, 8, 14): a wave then runs lines of one length, where interleaved lengths made every
// lane pay for every filter variant of its wave.  Order within a group is free (edges of one direction never overlap).
// Returns the count; list[] holds record indices.  Ends with a barrier.
__device__ __forceinline__ int list_edges(const uint32_t *rec, int n, const uint8_t *lvl, uint16_t *list, int *s_cnt) {
    const int tid = threadIdx.x, lane = tid & 63;
    auto bucket = [&](int ri) {
        const uint32_t r   = rec[ri];
        const int      len = r & 15;
        if (!len || (!lvl[(r >> 8) & 127] && !lvl[(r >> 16) & 127])) return -1;
        return len == 4 ? 0 : len == 6 ? 1 : len == 8 ? 2 : 3;
    };
    if (tid < 8) s_cnt[tid] = 0; // [0, 4): counts, then cursors; [4, 8): group starts
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += NTHR) {
        const int b = i0 + tid < n ? bucket(i0 + tid) : -1;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const unsigned long long m = __ballot(b == g);
            if (m && lane == __ffsll((long long)m) - 1) atomicAdd(&s_cnt[g], (int)__popcll(m));
        }
    }
    __syncthreads();
    if (tid == 0) {
        int o = 0;
        for (int g = 0; g < 4; g++) {
            const int c = s_cnt[g];
            s_cnt[4 + g] = o, s_cnt[g] = o, o += c;
        }
    }
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += NTHR) {
        const int b = i0 + tid < n ? bucket(i0 + tid) : -1;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const unsigned long long m = __ballot(b == g);
            if (!m) continue;
            const int leader = __ffsll((long long)m) - 1;
            int       base   = 0;
            if (lane == leader) base = atomicAdd(&s_cnt[g], (int)__popcll(m));
            base = __shfl(base, leader);
            if (b == g) list[base + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)(i0 + tid);
        }
    }
    __syncthreads();
    return s_cnt[3]; // the last group's cursor ends at the total
}

// one (plane job, tile, trial) item -- item `bi` of `nbi` -- of a trial or apply launch (uniform per workgroup)
template <typename T, bool TRIAL>
__device__ __forceinline__ void dlf_tile_item(KArgs &a, int bi, int nbi, DlfTileLds &L) {
    uint16_t           *t = L.t;
    uint32_t           *rv = L.rv, *rh = L.rh;
    unsigned long long *red = L.red;
    uint8_t(*s_lvl)[128]   = L.s_lvl;
    uint32_t           *s_thr = L.s_thr;
    uint16_t           *s_list = L.s_list;
    int                *s_cnt = L.s_cnt;
    const int           tid = threadIdx.x;
    wgclk_mark(a.wgclk, 0);
    // one (plane job, tile, trial) per item: the trials of a tile are neighbours after the XCD swizzle, so the second
    // staging of a tile hits the L2; one working image in LDS (18 KB) keeps 8 waves per SIMD.  a.dyn: the items are the
    // device plan's levels only (its trial count per job), no item for an untried level
    const int b = xcd_swizzle(bi, nbi);
#define DLF_NTR(j) (TRIAL ? (a.dyn ? a.plan->ntrial[j] : a.job[j].ntrial) : 1)
    int       jb = 0, tb = b;
    while (jb + 1 < a.njob && tb >= a.job[jb].tiles * DLF_NTR(jb)) tb -= a.job[jb].tiles * DLF_NTR(jb), jb++;
    KJob     &J  = a.job[jb];
    const int nt = DLF_NTR(jb);
#undef DLF_NTR
    if (TRIAL && nt == 0) return;
    const int tr = TRIAL ? tb % nt : 0;
    if (TRIAL) tb /= nt;
    if (TRIAL && a.plan && tr >= a.plan->ntrial[jb]) return; // a level the device plan does not try this launch
    const int x0 = J.ox + (tb % J.tiles_x) * TILE, y0 = J.oy + (tb / J.tiles_x) * TILE;
    const int gx = x0 - APRON, gy = y0 - APRON;
    const T  *src = (const T *)J.src;
    __syncthreads(); // this workgroup's previous item is done with the LDS
    s_lvl[tid >> 7][tid & 127] = (TRIAL && a.plan) ? a.plan->lvl[jb][tr][tid >> 7][tid & 127]
                               : (!TRIAL && a.dev_lvl) ? a.dev_lvl[(J.plane * 2 + (tid >> 7)) * 128 + (tid & 127)]
                                                       : J.lvl[tr][tid >> 7][tid & 127]; // NTHR == 256 entries
    if (tid < 64) s_thr[tid] = (uint32_t)a.mblim[tid] | ((uint32_t)a.lim[tid] << 8) | ((uint32_t)a.hev[tid] << 16);

    // edge records reaching the tile (no records outside the plane: length 0) and the tile + apron (samples outside
    // the plane are never read by an active edge), 4 samples per item (gx is a multiple of 4: aligned 8-B / 4-B
    // loads); every load of a lane is issued before the first LDS store
    constexpr int RV_R = LW / 4, RV_C = TILE / 4 + 3, RH_R = TILE / 4 + 3, RH_C = TILE / 4;
    constexpr int NV = RV_R * RV_C, NH = RH_R * RH_C, IR = (NV + NTHR - 1) / NTHR, IH = (NH + NTHR - 1) / NTHR;
    constexpr int NS = LW * LW / 4, IS = (NS + NTHR - 1) / NTHR;
    uint32_t      vrec[IR], hrec[IH];
    uint2         q[IS];
#pragma unroll
    for (int u = 0; u < IR; u++) {
        const int i = tid + u * NTHR, ur = gy / 4 + i / RV_C, uc = (x0 - 4) / 4 + i % RV_C;
        vrec[u] = (i < NV && ur >= 0 && uc >= 0 && ur * 4 < J.ph && uc * 4 < J.pw) ? J.rec_v[(size_t)ur * J.units_w + uc] : 0u;
    }
#pragma unroll
    for (int u = 0; u < IH; u++) {
        const int i = tid + u * NTHR, ur = (y0 - 4) / 4 + i / RH_C, uc = x0 / 4 + i % RH_C;
        hrec[u] = (i < NH && ur >= 0 && ur * 4 < J.ph && uc * 4 < J.pw) ? J.rec_h[(size_t)ur * J.units_w + uc] : 0u;
    }
#pragma unroll
    for (int u = 0; u < IS; u++) {
        const int i = tid + u * NTHR, r = gy + i / (LW / 4), c = gx + 4 * (i % (LW / 4));
        q[u] = make_uint2(0u, 0u);
        if (i >= NS || r < 0 || r >= J.ph) continue;
        const T *sp = src + (size_t)r * J.src_stride + c;
        if (c >= 0 && c + 4 <= J.pw) {
            if constexpr (sizeof(T) == 2) {
                q[u] = *(const uint2 *)sp;
            } else {
                const uint32_t b = *(const uint32_t *)sp;
                q[u] = make_uint2((b & 0xFF) | ((b & 0xFF00) << 8), ((b >> 16) & 0xFF) | ((b >> 8) & 0xFF0000));
            }
        } else {
            uint32_t w[2] = {0u, 0u};
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (c + j >= 0 && c + j < J.pw) w[j >> 1] |= (uint32_t)(uint16_t)sp[j] << (16 * (j & 1));
            q[u] = make_uint2(w[0], w[1]);
        }
    }
#pragma unroll
    for (int u = 0; u < IR; u++)
        if (tid + u * NTHR < NV) rv[tid + u * NTHR] = vrec[u];
#pragma unroll
    for (int u = 0; u < IH; u++)
        if (tid + u * NTHR < NH) rh[tid + u * NTHR] = hrec[u];
#pragma unroll
    for (int u = 0; u < IS; u++)
        if (tid + u * NTHR < NS) *(uint2 *)&t[4 * (tid + u * NTHR)] = q[u];
    const int tw = min(TILE, J.ox + J.ow - x0), th = min(TILE, J.oy + J.oh - y0);
    {
        __syncthreads();
        wgclk_mark(a.wgclk, 1);
        // vertical edges x0-4 .. x0+64 over all 88 rows: (listed edge, line) per item
        const int nve = list_edges(rv, NV, s_lvl[0], s_list, s_cnt);
        for (int i = tid; i < ((DLF_EXP & 1) ? 0 : nve * 4); i += NTHR) {
            const int ri = s_list[i >> 2], line = i & 3, e = ri % RV_C, sr = ri / RV_C;
            const uint32_t r = rv[ri];
            const int len = r & 15;
            const int cur = s_lvl[0][(r >> 8) & 127], prv = s_lvl[0][(r >> 16) & 127];
            const uint32_t th = s_thr[cur ? cur : prv];
            uint16_t *row = &t[(sr * 4 + line) * LW + (APRON - 4 + e * 4)];
            const int h = half_taps(len);
            int F[14];
#pragma unroll
            for (int k = 0; k < 14; k++) F[k] = (k >= 7 - h && k < 7 + h) ? row[k - 7] : 0;
            filter_line(F, len, th & 0xFF, (th >> 8) & 0xFF, th >> 16, a.bd);
#pragma unroll
            for (int k = 0; k < 14; k++)
                if (k >= 7 - h && k < 7 + h) row[k - 7] = (uint16_t)F[k];
        }
        __syncthreads();
        wgclk_mark(a.wgclk, 2);
        // horizontal edges y0-4 .. y0+64 over the tile's 64 columns: (listed 4-column edge segment, column) per item
        const int nhe = list_edges(rh, NH, s_lvl[1], s_list, s_cnt);
        for (int i = tid; i < ((DLF_EXP & 2) ? 0 : nhe * 4); i += NTHR) {
            const int ri = s_list[i >> 2], e = ri / RH_C, col = 4 * (ri % RH_C) + (i & 3);
            const uint32_t r = rh[ri];
            const int len = r & 15;
            const int cur = s_lvl[1][(r >> 8) & 127], prv = s_lvl[1][(r >> 16) & 127];
            const uint32_t th = s_thr[cur ? cur : prv];
            uint16_t *c = &t[(APRON - 4 + e * 4) * LW + APRON + col];
            const int h = half_taps(len);
            int F[14];
#pragma unroll
            for (int k = 0; k < 14; k++) F[k] = (k >= 7 - h && k < 7 + h) ? c[(k - 7) * LW] : 0;
            filter_line(F, len, th & 0xFF, (th >> 8) & 0xFF, th >> 16, a.bd);
#pragma unroll
            for (int k = 0; k < 14; k++)
                if (k >= 7 - h && k < 7 + h) c[(k - 7) * LW] = (uint16_t)F[k];
        }
        __syncthreads();
        wgclk_mark(a.wgclk, 3);
        // emit the tile
        if (TRIAL) {
            uint32_t  s = 0; // <= 16 samples per lane
            const T  *ref = (const T *)J.ref;
            const int c = tid % TILE;
            if (c < tw) {
                int rv16[TILE / (NTHR / TILE)]; // the lane's source samples, all loads in flight together
#pragma unroll
                for (int k = 0; k < TILE / (NTHR / TILE); k++) {
                    const int r = tid / TILE + k * (NTHR / TILE);
                    rv16[k] = r < th ? (int)ref[(size_t)(y0 + r) * J.ref_stride + x0 + c] : 0;
                }
#pragma unroll
                for (int k = 0; k < TILE / (NTHR / TILE); k++) {
                    const int r = tid / TILE + k * (NTHR / TILE);
                    const int d = r < th ? (int)t[(APRON + r) * LW + APRON + c] - rv16[k] : 0;
                    s += (uint32_t)(d * d);
                }
            }
            const unsigned long long sw = wave_sum_u32_wide(s);
            if ((tid & 63) == 63) red[tid >> 6] = sw;
            __syncthreads();
            if (tid == 0) {
                unsigned long long tot = 0;
                for (int w = 0; w < NTHR / 64; w++) tot += red[w];
                atomicAdd(&a.sse[jb * MAX_TRIALS + tr], tot);
            }
        } else {
            // 4 samples per item: x0 is a multiple of 64 and tw of 4, so every item is whole and aligned
            T *dst = (T *)J.dst;
            for (int i = tid; i < TILE * TILE / 4; i += NTHR) {
                const int r = i / (TILE / 4), c = 4 * (i % (TILE / 4));
                if (r >= th || c >= tw) continue;
                const uint2 w = *(const uint2 *)&t[(APRON + r) * LW + APRON + c];
                T *d = dst + (size_t)(y0 + r) * J.dst_stride + x0 + c;
                if constexpr (sizeof(T) == 2)
                    *(uint2 *)d = w;
                else
                    *(uint32_t *)d = (w.x & 0xFF) | ((w.x >> 8) & 0xFF00) | ((w.y & 0xFF) << 16) | ((w.y & 0xFF0000) << 8);
            }
        }
    }
    wgclk_mark(a.wgclk, 5);
}

template <typename T, bool TRIAL>
__global__ __launch_bounds__(NTHR, 8) void dlf_tile_kernel(const DlfTileArgs a0) {
    __shared__ __align__(16) DlfTileLds L;
    KArgs    &a   = kargs();
    const int tid = threadIdx.x;
    dlf_tile_item<T, TRIAL>(a, blockIdx.x, gridDim.x, L);
    // trial: the last workgroup to finish reads the sums (8-B agent atomics on both sides; this lane's SSE adds have
    // completed before its arrival is counted) and re-arms the accumulators for the next launch
    if (TRIAL && tid == 0 && !a.plan) { // (device plan: dlf_search_step_kernel reads the sums in stream order)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (atomicAdd(a.arrive, 1u) == gridDim.x - 1) {
            for (int q = 0; q < MAX_JOBS * MAX_TRIALS; q++) a.out[q] = atomicExch(&a.sse[q], 0ull);
            atomicExch(a.arrive, 0u);
            __threadfence_system(); // the sums reach the host before the word that announces them
            __hip_atomic_store(&a.out[MAX_JOBS * MAX_TRIALS], a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// plane SSE (svt_spatial_full_distortion_kernel / svt_full_distortion_kernel16_bits)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void plane_sse_kernel(const T *a, int as, const T *b, int bs, int w, int h,
                                                        unsigned long long *out) {
    __shared__ unsigned long long red[4];
    unsigned long long s = 0;
    for (int r = blockIdx.x; r < h; r += gridDim.x)
        for (int c = threadIdx.x; c < w; c += 256) {
            const int d = (int)a[(size_t)r * as + c] - (int)b[(size_t)r * bs + c];
            s += (unsigned long long)(d * d);
        }
    s = wave_sum_lane63(s);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

// ---------------------------------------------------------------------------------------------
// per-segment shim kernel: 4 lines of one edge, staged as [4][16] with the edge between 7 and 8
// ---------------------------------------------------------------------------------------------
__global__ void lpf_lines_kernel(uint16_t *lines, int len, int blimit, int limit, int thresh, int bd) {
    const int l = threadIdx.x;
    if (l >= 4) return;
    int F[14];
    for (int k = 0; k < 14; k++) F[k] = lines[l * 16 + 1 + k];
    filter_line(F, len, blimit, limit, thresh, bd);
    for (int k = 0; k < 14; k++) lines[l * 16 + 1 + k] = (uint16_t)F[k];
}

} // namespace

// =============================================================================================
// host side
// =============================================================================================
struct SvtGpuDlfState {
    SvtGpuContext *ctx;
    int32_t        width, height, mi_rows, mi_cols;
    SvtGpuLfMi    *d_mi;
    uint32_t      *d_rec[2][2]; // [chroma][dir]
    int32_t        uw[2], uh[2]; // record grid per plane type
    int32_t        crop_w, crop_h; // the unpadded luma size (svtgpu_dlf_set_crop; default the coded size)
    void          *d_scratch;    // plane copy for in-place apply
    unsigned long long *d_sse;   // trial accumulators [MAX_JOBS][MAX_TRIALS], zero between launches
    unsigned int       *d_arrive; // trial workgroup arrivals, zero between launches
    unsigned long long *h_sse;   // pinned, mapped: the trial results written by the kernel's last workgroup
    unsigned long long *h_sse_dev; // its device address
    unsigned long long  seq;       // last trial launch's sequence number
    int32_t        have_mi;
    int32_t        mi_on_device = 0; // the last grid came through svtgpu_dlf_set_mode_info_device (checked there)
    // frame tiling over GPUs (svtgpu_dlf_set_tile): trial SSEs over sse_rect, summed over `comm`; the apply writes
    // out_rect (luma {x0, y0, x1, y1}; the whole frame by default)
    int32_t        sse_rect[4] = {0, 0, 0, 0}, out_rect[4] = {0, 0, 0, 0};
    SvtGpuComm    *comm = nullptr;
    void          *d_search = nullptr;  // DlfDevSearch: the device-resident level search (SVTGPU_DLF_DEVICE)
    void          *d_plans  = nullptr;  // DlfDevPlan[2]: the asynchronous search's trial launches read plan k & 1
    void          *h_search = nullptr;  // its pinned host copy
    SvtGpuLfMi    *h_mi = nullptr;      // pinned staging of the mode info (one upload per frame, asynchronous)
    SvtGpuPrioLane prio;                // the level search's trial launches
    hipEvent_t     mi_free = nullptr;   // the previous upload has read h_mi
    // svtgpu_dlf_pick_async: the result the device search leaves (device: the apply's tables; mapped: the caller's
    // levels), the picks enqueued / collected, the parameters it started from, the rounds to enqueue next time
    void          *d_res = nullptr, *h_res = nullptr, *h_res_dev = nullptr;
    int32_t        dev_seq = 0, dev_pending = 0, dev_ready = 0, dev_rounds = 8, dev_rounds_last = 0, dev_seen = 0;
    SvtGpuLfParams dev_params{};
};

namespace {

// level tables: svt_av1_loop_filter_frame_init + svt_aom_update_sharpness (EbDeblockingCommon.c:76-139, 554-572)
struct LevelTables {
    uint8_t lvl[3][2][128]; // [plane][dir][segment*16 + ref*2 + mode_lf]
    uint8_t mblim[64], lim[64], hev[64];
};

__host__ __device__ static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

// the level per (segment, reference, mode) class of one plane and direction whose base level is lv
// (svt_av1_loop_filter_frame_init, EbDeblockingFilter.c)
// one (segment, reference, mode) class of it: cls = seg * 16 + ref * 2 + mode
__host__ __device__ static inline uint8_t level_entry(const SvtGpuLfParams &p, int pl, int dir, int lv, int cls) {
    const int feat[3][2] = {{1, 2}, {3, 3}, {4, 4}}; // SEG_LVL_ALT_LF_{Y_V, Y_H, U, V}
    const int seg = cls >> 4, ref = (cls >> 1) & 7, mode = cls & 1;
    int       ls  = lv;
    if (p.segmentation_enabled && p.seg_feature_enabled[seg][feat[pl][dir]])
        ls = clampi(ls + p.seg_feature_data[seg][feat[pl][dir]], 0, 63);
    int v = ls;
    if (p.mode_ref_delta_enabled) {
        const int scale = 1 << (ls >> 5);
        v = ls + p.ref_deltas[ref] * scale + (ref > 0 ? p.mode_deltas[mode] * scale : 0);
        v = clampi(v, 0, 63);
    }
    return (uint8_t)v;
}

__host__ __device__ static void fill_level_table(const SvtGpuLfParams &p, int pl, int dir, int lv, uint8_t *out) {
    for (int cls = 0; cls < 128; cls++) out[cls] = level_entry(p, pl, dir, lv, cls);
}

void build_level_tables(const SvtGpuLfParams &p, LevelTables &L) {
    std::memset(&L, 0, sizeof L);
    const int sh = p.sharpness_level;
    for (int l = 0; l < 64; l++) {
        int inside = l >> ((sh > 0) + (sh > 4));
        if (sh > 0) inside = std::min(inside, 9 - sh);
        inside     = std::max(inside, 1);
        L.lim[l]   = (uint8_t)inside;
        L.mblim[l] = (uint8_t)(2 * (l + 2) + inside);
        L.hev[l]   = (uint8_t)(l >> 4);
    }
    const int base[3][2] = {{p.filter_level[0], p.filter_level[1]},
                            {p.filter_level_u, p.filter_level_u},
                            {p.filter_level_v, p.filter_level_v}};
    for (int pl = 0; pl < 3; pl++)
        for (int dir = 0; dir < 2; dir++) fill_level_table(p, pl, dir, base[pl][dir], L.lvl[pl][dir]);
}

// is the plane filtered at all with these levels (svt_aom_loop_filter_sb :575-582)
__host__ __device__ bool plane_active(const SvtGpuLfParams &p, int plane) {
    if (plane == 0) return p.filter_level[0] || p.filter_level[1];
    return plane == 1 ? p.filter_level_u != 0 : p.filter_level_v != 0;
}

DlfPlaneJob plane_job(SvtGpuDlfState *s, const SvtGpuFrame *f, int plane, bool trial) {
    DlfPlaneJob j;
    std::memset(&j, 0, sizeof j);
    j.plane   = plane;
    const int ch = plane > 0;
    j.rec_v   = s->d_rec[ch][0];
    j.rec_h   = s->d_rec[ch][1];
    j.units_w = s->uw[ch];
    j.pw      = f->pw[plane];
    j.ph      = f->ph[plane];
    // trials measure the SSE rectangle, the apply writes the output rectangle (luma coordinates; chroma halved,
    // rounded outward); both the whole plane unless a tile is set
    const int32_t *r = trial ? s->sse_rect : s->out_rect;
    const int      sh = plane > 0;
    j.ox      = r[0] >> sh, j.oy = r[1] >> sh;
    j.ow      = std::min(j.pw, (r[2] + sh) >> sh) - j.ox, j.oh = std::min(j.ph, (r[3] + sh) >> sh) - j.oy;
    j.tiles_x = (j.ow + TILE - 1) / TILE;
    j.tiles   = j.ow > 0 && j.oh > 0 ? j.tiles_x * ((j.oh + TILE - 1) / TILE) : 0;
    return j;
}

DlfTileArgs base_args(const SvtGpuFrame *f, const LevelTables &L) {
    DlfTileArgs a;
    std::memset(&a, 0, sizeof a);
    a.bd = f->bit_depth;
    std::memcpy(a.mblim, L.mblim, 64);
    std::memcpy(a.lim, L.lim, 64);
    std::memcpy(a.hev, L.hev, 64);
    return a;
}

int launch_tile(const DlfTileArgs &a0, int bps, bool trial, hipStream_t st) {
    int tiles = 0; // workgroups: one per tile (apply) or per (tile, trial)
    for (int j = 0; j < a0.njob; j++) tiles += a0.job[j].tiles * (trial ? a0.job[j].ntrial : 1);
    DlfTileArgs a = a0;
    a.wgclk       = svtgpu_wgclk_begin(tiles);
    if (bps == 2) {
        if (trial) hipLaunchKernelGGL((dlf_tile_kernel<uint16_t, true>), dim3(tiles), dim3(NTHR), 0, st, a);
        else       hipLaunchKernelGGL((dlf_tile_kernel<uint16_t, false>), dim3(tiles), dim3(NTHR), 0, st, a);
    } else {
        if (trial) hipLaunchKernelGGL((dlf_tile_kernel<uint8_t, true>), dim3(tiles), dim3(NTHR), 0, st, a);
        else       hipLaunchKernelGGL((dlf_tile_kernel<uint8_t, false>), dim3(tiles), dim3(NTHR), 0, st, a);
    }
    HIP_TRY(hipGetLastError());
    svtgpu_wgclk_end(trial ? "dlf_trial" : "dlf_apply", tiles, st);
    return SVTGPU_OK;
}

bool frame_matches(const SvtGpuDlfState *s, const SvtGpuFrame *f) {
    return f && f->width == s->width && f->height == s->height && (f->bit_depth == 8 || f->bit_depth == 10);
}

__host__ __device__ void set_trial_level(SvtGpuLfParams &p, int plane, int dir, int lvl) { // try_filter_frame (:841-883)
    if (plane == 0) {
        if (dir != 1) p.filter_level[0] = lvl;
        if (dir != 0) p.filter_level[1] = lvl;
    } else if (plane == 1)
        p.filter_level_u = lvl;
    else
        p.filter_level_v = lvl;
}

// search_filter_level (EbDeblockingFilter.c:886-991) as a resumable state machine: pending() names the levels the
// next step needs (advancing over steps whose levels are already known), feed() records their SSE.  Independent
// searches (U and V) then share launches.
struct LevelSearch {
    int     plane = 0, dir = 0, early_exit = 0, only4x4 = 0;
    int     mid = 0, step = 0, direction = 0, conv = 0, best = 0;
    int64_t best_err = 0, bias = 0, err[64];
    int     phase = 0; // 0: the start level; 1: bisection steps; 2: done
    int     lo = 0, hi = 0;
    bool    try_lo = false, try_hi = false;
    int     req[MAX_TRIALS], nreq = 0;

    __host__ __device__ LevelSearch() {}
    __host__ __device__ LevelSearch(const int last[4], int dlf_avg, int early_exit_, int only4x4_, int plane_, int dir_)
        : plane(plane_), dir(dir_), early_exit(early_exit_), only4x4(only4x4_) {
        const int start = plane == 0 ? (dlf_avg ? last[0] : last[dir]) : last[plane + 1];
        mid  = clampi(start, 0, 63);
        step = mid < 16 ? 4 : mid / 4;
        best = mid;
        for (int i = 0; i < 64; i++) err[i] = -1;
        req[0] = mid, nreq = 1;
    }
    // the next bisection step's candidates (try lo / hi around mid), or done
    __host__ __device__ void next_request() {
        if (step <= 0) {
            phase = 2, nreq = 0;
            return;
        }
        hi   = mid + step < 63 ? mid + step : 63, lo = mid - step > 0 ? mid - step : 0;
        bias = (best_err >> (15 - (mid / 8))) * step;
        if (!only4x4) bias >>= 1;
        try_lo = direction <= 0 && lo != mid, try_hi = direction >= 0 && hi != mid;
        nreq   = 0;
        if (try_lo) req[nreq++] = lo;
        if (try_hi) req[nreq++] = hi;
    }
    __host__ __device__ void resolve() {
        if (phase == 0) {
            best_err = err[mid], best = mid, phase = 1;
        } else {
            if (try_lo && err[lo] < best_err + bias) {
                if (err[lo] < best_err) best_err = err[lo];
                best = lo;
            }
            if (try_hi && err[hi] < best_err - bias) {
                best_err = err[hi];
                best     = hi;
            }
            if (best == mid) {
                conv++;
                step      = conv == early_exit ? 0 : step / 2;
                direction = 0;
            } else {
                direction = best < mid ? -1 : 1;
                mid       = best;
            }
        }
        next_request();
    }
    __host__ __device__ int pending(int *lv) {
        while (phase != 2) {
            int m = 0;
            for (int k = 0; k < nreq; k++) {
                bool dup = err[req[k]] >= 0;
                for (int j = 0; j < m && !dup; j++) dup = lv[j] == req[k];
                if (!dup) lv[m++] = req[k];
            }
            if (m) return m;
            resolve();
        }
        return 0;
    }
    __host__ __device__ void feed(const int *lv, int m, const unsigned long long *sse) {
        for (int k = 0; k < m; k++) err[lv[k]] = (int64_t)sse[k];
    }
};

// The device-resident form of the searches (SVTGPU_DLF_DEVICE=1): the plane searches, the frame's parameters and the
// next trial launch's plan live in HBM; after each trial launch one single-lane kernel feeds the SSEs to the searches
// and writes the next plan, so the bisection advances with no host decision between trials.  The host enqueues a
// chunk of (trial, step) pairs and reads the state back once per chunk; launches after the searches have finished
// find an empty plan (every workgroup returns at once).
struct DlfDevSearch {
    LevelSearch    srch[MAX_JOBS];
    int32_t        ns;
    SvtGpuLfParams p;
    DlfDevPlan     plan;
    int32_t        rounds; // trial rounds taken (svtgpu_dlf_pick_async)
};
// what an asynchronous search leaves for the apply (device) and the caller (mapped host memory)
struct DlfDevResult {
    int32_t levels[4]; // filter_level[0], [1], _u, _v
    int32_t rounds, seq, pad[2];
    uint8_t lvl[3][2][128]; // the apply's level tables of the picked levels (zero for a plane that is not filtered)
};

// the next launch's levels per search (the bisection steps), then each (search, level)'s tables: that plane's only, as
// run_searches builds them (try_filter_frame sets one plane's level; the other levels and the class deltas stay)
__host__ __device__ void plan_levels(DlfDevSearch &S) {
    S.plan.done = 1;
    for (int i = 0; i < MAX_JOBS; i++) {
        const int m = i < S.ns ? S.srch[i].pending(S.plan.lv[i]) : 0;
        S.plan.ntrial[i] = m;
        if (m) S.plan.done = 0;
    }
}
// table entry e of [MAX_JOBS][MAX_TRIALS][2][128] (entries of levels the plan does not try are left as they are)
__host__ __device__ inline void plan_table_entry(DlfDevSearch &S, int e) {
    const int cls = e & 127, d = (e >> 7) & 1, k = (e >> 8) % MAX_TRIALS, i = (e >> 8) / MAX_TRIALS;
    if (i >= S.ns || k >= S.plan.ntrial[i]) return;
    const int plane = S.srch[i].plane, lvl = S.plan.lv[i][k];
    int       l0 = S.p.filter_level[0], l1 = S.p.filter_level[1], lu = S.p.filter_level_u, lvv = S.p.filter_level_v;
    if (plane == 0) { // set_trial_level
        if (S.srch[i].dir != 1) l0 = lvl;
        if (S.srch[i].dir != 0) l1 = lvl;
    } else if (plane == 1)
        lu = lvl;
    else
        lvv = lvl;
    const bool on   = plane == 0 ? (l0 || l1) : plane == 1 ? lu != 0 : lvv != 0; // plane_active
    const int  base = plane == 0 ? (d == 0 ? l0 : l1) : plane == 1 ? lu : lvv;
    S.plan.lvl[i][k][d][cls] = on ? level_entry(S.p, plane, d, base, cls) : 0;
}
constexpr int PLAN_ENTRIES = MAX_JOBS * MAX_TRIALS * 2 * 128;
void plan_next(DlfDevSearch &S) { // host
    plan_levels(S);
    for (int e = 0; e < PLAN_ENTRIES; e++) plan_table_entry(S, e);
}

// one bisection decision per search from the last trial launch's sums (re-zeroed), then the next plan.  The state is
// copied into the LDS words `w` (>= sizeof(DlfDevSearch) / 4) by the workgroup and walked there by one lane (the
// search is a chain of dependent reads: from global memory each would wait a full memory latency), then written back.
// atomic_sums: the sums are exchanged to zero with device-scope atomics (a workgroup of the trial launch itself runs
// the step), else read and zeroed in stream order
static_assert(sizeof(DlfDevSearch) % 4 == 0, "word copies of the search state");
static_assert(sizeof(DlfDevSearch) <= sizeof(DlfTileLds::t), "the step's LDS copy fits the tile image it reuses");
// out_plan (nullable): the plan buffer the next trial launch reads (the asynchronous search's double-buffered plans)
__device__ void copy_plan(DlfDevPlan *dst, const DlfDevPlan *src) {
    constexpr int NP = (int)(sizeof(DlfDevPlan) / 4);
    for (int i = threadIdx.x; i < NP; i += blockDim.x) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
}
__device__ void dlf_step(DlfDevSearch *S, unsigned long long *sse, uint32_t *w, bool atomic_sums,
                         DlfDevPlan *out_plan = nullptr) {
    constexpr int NW = (int)(sizeof(DlfDevSearch) / 4);
    const int     tid = threadIdx.x, nt = blockDim.x;
    for (int i = tid; i < NW; i += nt) w[i] = ((const uint32_t *)S)[i];
    __syncthreads();
    DlfDevSearch &D = *(DlfDevSearch *)w;
    if (D.plan.done) { // uniform: every lane read the same word
        if (out_plan) copy_plan(out_plan, &D.plan);
        return;
    }
    __shared__ unsigned long long v[MAX_JOBS * MAX_TRIALS]; // the sums, one lane each (not a chain of atomics)
    if (tid < MAX_JOBS * MAX_TRIALS) v[tid] = atomic_sums ? atomicExch(&sse[tid], 0ull) : sse[tid];
    __syncthreads();
    if (tid == 0) {
        for (int i = 0; i < D.ns; i++)
            if (D.plan.ntrial[i]) D.srch[i].feed(D.plan.lv[i], D.plan.ntrial[i], v + i * MAX_TRIALS);
        plan_levels(D);
        D.rounds++;
    }
    __syncthreads();
    for (int e = tid; e < PLAN_ENTRIES; e += nt) plan_table_entry(D, e); // the tables: one entry per lane and pass
    __syncthreads();
    if (!atomic_sums && tid < MAX_JOBS * MAX_TRIALS) sse[tid] = 0;
    for (int i = tid; i < NW; i += nt) ((uint32_t *)S)[i] = w[i];
    if (out_plan) copy_plan(out_plan, &D.plan);
}
__global__ __launch_bounds__(64) void dlf_search_step_kernel(DlfDevSearch *S, unsigned long long *sse) {
    __shared__ __align__(16) uint32_t w[sizeof(DlfDevSearch) / 4];
    dlf_step(S, sse, w, false);
}

// svtgpu_dlf_pick_async, 1: the searches' start (LevelSearch's constructor: the start level) and the first plan,
// from the caller's parameters -- no host staging
__global__ __launch_bounds__(64) void dlf_search_init_kernel(DlfDevSearch *S, SvtGpuLfParams p, int ns, int dlf_avg,
                                                            int early_exit, int only4x4) {
    __shared__ __align__(16) uint32_t w[sizeof(DlfDevSearch) / 4];
    constexpr int NW = (int)(sizeof(DlfDevSearch) / 4);
    DlfDevSearch &D  = *(DlfDevSearch *)w;
    const int     tid = threadIdx.x;
    if (tid == 0) {
        const int last[4] = {p.filter_level[0], p.filter_level[1], p.filter_level_u, p.filter_level_v};
        const int dirs[3] = {2, 0, 0};
        for (int i = 0; i < MAX_JOBS; i++) D.srch[i] = LevelSearch(last, dlf_avg, early_exit, only4x4, i, dirs[i]);
        D.ns = ns, D.p = p, D.rounds = 0;
        plan_levels(D);
    }
    __syncthreads();
    for (int e = tid; e < PLAN_ENTRIES; e += 64) plan_table_entry(D, e);
    __syncthreads();
    for (int i = tid; i < NW; i += 64) ((uint32_t *)S)[i] = w[i];
}

// svtgpu_dlf_pick_async, 2: one trial round of the device plan (items = the plan's levels only);
// the last workgroup to finish takes the bisection step (fuse; a tiled rank steps after the SSE all-reduce instead)
template <typename T>
__global__ __launch_bounds__(NTHR, 8) void dlf_trial_dev_kernel(const DlfTileArgs a0, DlfDevSearch *S, int fuse) {
    __shared__ __align__(16) DlfTileLds L;
    KArgs    &a = kargs();
    __shared__ int last;
    const int tid    = threadIdx.x;
    int       nitems = 0;
    // This launch reads its own plan buffer (a.plan = plan k & 1), which nothing writes while it runs: the step of the
    // round writes the NEXT launch's buffer (next_plan).  A spare workgroup dispatched late (behind other frames'
    // kernels, after the step) therefore still reads this round's plan.  (With one plan rewritten in place, such a
    // workgroup could read the next round's plan, take one of its items and arrive at the freshly reset counter: the
    // next round's step fired one arrival early and every later round of that state stayed off by one -- round 6,
    // one frame slot's DLF stage at 41 ms per frame under load.)
    for (int j = 0; j < a.njob; j++) nitems += a.job[j].tiles * a.plan->ntrial[j];
    if (nitems == 0) { // every search has finished: carry the finished plan to the next launch's buffer
        if (fuse && a.next_plan && blockIdx.x == 0) copy_plan(a.next_plan, a.plan);
        return;
    }
    // one item per workgroup over a grid sized for the most levels a round can try; the workgroups past this round's
    // items go straight out, uncounted (a persistent loop over the items spilled 60 VGPRs: the item's registers live
    // across the loop)
    if ((int)blockIdx.x >= nitems) return;
    dlf_tile_item<T, true>(a, blockIdx.x, nitems, L);
    if (!fuse) return;
    __syncthreads();
    // No __threadfence: an agent-scope fence writes back and invalidates this XCD's L2 (the L2s of the 8 XCDs are not
    // coherent), which doubled every round (the trials of a tile share their staging through the L2); the sums are
    // device-scope atomics, so waiting for this lane's to complete before its arrival is enough
    if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(a.arrive, 1u) == (unsigned)nitems - 1;
    }
    __syncthreads();
    if (!last) return;
    dlf_step(S, a.sse, (uint32_t *)L.t, true, a.next_plan);
    if (tid == 0) atomicExch(a.arrive, 0u);
}

// svtgpu_dlf_pick_async, 3: one workgroup.  A search still unfinished after the enqueued rounds (they are sized from the
// previous frame's count) continues here, exactly, each round's items looped by this workgroup alone -- slow, but no
// host decision; then the apply's level tables of the picked levels and the caller's result (mapped memory)
template <typename T>
__global__ __launch_bounds__(NTHR) void dlf_finish_kernel(const DlfTileArgs a0, DlfDevSearch *S, DlfDevResult *res,
                                                          DlfDevResult *host, int seq) {
    __shared__ __align__(16) DlfTileLds L;
    KArgs    &a = kargs();
    __shared__ int done;
    const int tid = threadIdx.x;
    for (int guard = 0; guard < 4096; guard++) { // a search ends after at most ~64 rounds
        if (tid == 0) done = __hip_atomic_load(&S->plan.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (done) break;
        int nitems = 0;
        for (int j = 0; j < a.njob; j++) nitems += a.job[j].tiles * a.plan->ntrial[j];
        for (int i = 0; i < nitems; i++) dlf_tile_item<T, true>(a, i, nitems, L);
        __syncthreads();
        if (tid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the last item's SSE atomic
        __syncthreads();
        dlf_step(S, a.sse, (uint32_t *)L.t, true);
        __syncthreads();
    }
    // the picked levels (svt_av1_pick_filter_level: luma both directions from the dir-2 search; chroma searched, or the
    // start levels when dlf_avg_uv skips it) and their tables (build_level_tables / plane_active / luma_off)
    __shared__ int lv[4];
    if (tid == 0) {
        const DlfDevSearch &D = *S;
        lv[0] = lv[1] = D.srch[0].best;
        lv[2] = D.ns == 3 ? D.srch[1].best : D.p.filter_level_u;
        lv[3] = D.ns == 3 ? D.srch[2].best : D.p.filter_level_v;
    }
    __syncthreads();
    SvtGpuLfParams q = S->p;
    q.filter_level[0] = lv[0], q.filter_level[1] = lv[1], q.filter_level_u = lv[2], q.filter_level_v = lv[3];
    const bool luma_off = !plane_active(q, 0);
    for (int e = tid; e < 3 * 2 * 128; e += NTHR) {
        const int pl = e >> 8, d = (e >> 7) & 1, cls = e & 127;
        const int base = pl == 0 ? q.filter_level[d] : pl == 1 ? q.filter_level_u : q.filter_level_v;
        res->lvl[pl][d][cls] = (!luma_off && plane_active(q, pl)) ? level_entry(q, pl, d, base, cls) : 0;
    }
    if (tid < 4) res->levels[tid] = lv[tid];
    if (tid == 0) {
        res->rounds = S->rounds, res->seq = seq;
        for (int k = 0; k < 4; k++) __hip_atomic_store(&host->levels[k], lv[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&host->rounds, S->rounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(&host->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// (trial, step) pairs per host read-back; 0: the host-driven search.  Default: the device search for a tile of a
// picture spread over ranks (its trial launches are small, so the host round trips and the all-reduce waits between
// them dominate: emulated 8-GPU rank 7.7-7.9 -> 8.1 Gpx/s), the host-driven one for a whole picture (its launches
// sized per step beat the device plan's full-shape grid: 3053 vs 2949 Mpx/s).  SVTGPU_DLF_DEVICE=0|1|n overrides.
int dlf_device_chunk(const SvtGpuDlfState *s) {
    static const int k = [] {
        const char *e = std::getenv("SVTGPU_DLF_DEVICE");
        return e ? std::max(0, std::min(64, std::atoi(e) == 1 ? 6 : std::atoi(e))) : -1;
    }();
    return k >= 0 ? k : (svtgpu_comm_tiled(s->comm) ? 6 : 0);
}

int run_searches_device_body(SvtGpuDlfState *s, const SvtGpuFrame *recon, const SvtGpuFrame *src,
                             const SvtGpuLfParams &p, LevelSearch *const *srch, int ns, hipStream_t st, int chunk) {
    if (!s->d_search) {
        HIP_TRY(hipMalloc(&s->d_search, sizeof(DlfDevSearch)));
        HIP_TRY(hipHostMalloc(&s->h_search, sizeof(DlfDevSearch), hipHostMallocDefault));
    }
    DlfDevSearch &H = *(DlfDevSearch *)s->h_search; // pinned: the caller's previous pick has read it back
    DlfDevSearch *D = (DlfDevSearch *)s->d_search;
    for (int i = 0; i < ns; i++) H.srch[i] = *srch[i];
    H.ns = ns;
    H.p  = p;
    plan_next(H);
    if (!H.plan.done) {
        HIP_TRY(hipMemcpyAsync(D, &H, sizeof H, hipMemcpyHostToDevice, st));
        svtgpu_count_xfer(0, sizeof H);
        LevelTables L;
        build_level_tables(p, L);
        DlfTileArgs a = base_args(recon, L);
        for (int i = 0; i < ns; i++) { // the grid covers MAX_TRIALS levels of every search; the plan says which run
            const int    plane = srch[i]->plane;
            DlfPlaneJob &J     = a.job[i];
            J                  = plane_job(s, recon, plane, true);
            J.src              = recon->plane[plane];
            J.src_stride       = recon->stride[plane];
            J.ref              = src->plane[plane];
            J.ref_stride       = src->stride[plane];
            J.ntrial           = MAX_TRIALS;
        }
        a.njob = ns;
        a.sse  = s->d_sse;
        a.plan = &D->plan;
        for (int launches = 0;;) {
            for (int k = 0; k < chunk; k++, launches++) {
                if (int rc = launch_tile(a, recon->bytes_per_sample, true, st)) return rc;
                // a picture tiled over GPUs: the frame's SSEs are the sums over the ranks (every rank then takes the
                // same decision)
                if (int rc = svtgpu_comm_sum(s->comm, s->d_sse, MAX_JOBS * MAX_TRIALS, true, st, SVTGPU_XCH_DLF)) return rc;
                hipLaunchKernelGGL(dlf_search_step_kernel, dim3(1), dim3(64), 0, st, D, s->d_sse);
                HIP_TRY(hipGetLastError());
            }
            HIP_TRY(hipMemcpyAsync(&H, D, sizeof H, hipMemcpyDeviceToHost, st));
            if (int rc = svtgpu_comm_wait(s->comm, st)) return rc; // bounded behind the SSE exchanges
            svtgpu_count_xfer(1, sizeof H);
            if (H.plan.done) break;
            if (launches >= 1024) { // a level search ends after far fewer trials
                svtgpu_set_last_hip_error(hipErrorUnknown, "dlf device level search: no convergence after 1024 trials",
                                          __FILE__, __LINE__);
                return SVTGPU_ERR_HIP;
            }
        }
    }
    for (int i = 0; i < ns; i++) *srch[i] = H.srch[i];
    return SVTGPU_OK;
}

// the device search; on any error exit the trial accumulators are zeroed again (the next pick assumes them zero)
int run_searches_device(SvtGpuDlfState *s, const SvtGpuFrame *recon, const SvtGpuFrame *src, const SvtGpuLfParams &p,
                        LevelSearch *const *srch, int ns, hipStream_t st, int chunk) {
    const int rc = run_searches_device_body(s, recon, src, p, srch, ns, st, chunk);
    if (rc) (void)hipMemsetAsync(s->d_sse, 0, sizeof(unsigned long long) * MAX_JOBS * MAX_TRIALS, st);
    return rc;
}

// run searches side by side: each launch evaluates the pending levels of every unfinished search (one plane job
// each), the SSE of every (job, level) comes back through mapped pinned memory; recon is never modified
int run_searches(SvtGpuDlfState *s, const SvtGpuFrame *recon, const SvtGpuFrame *src, const SvtGpuLfParams &p,
                 LevelSearch *const *srch, int ns, hipStream_t st) {
    for (;;) {
        DlfTileArgs a;
        int         lv[MAX_JOBS][MAX_TRIALS], m[MAX_JOBS], who[MAX_JOBS];
        bool        first = true;
        for (int i = 0; i < ns; i++) {
            const int mi = srch[i]->pending(lv[i]);
            if (!mi) continue;
            const int plane = srch[i]->plane;
            LevelTables L;
            if (first) {
                build_level_tables(p, L);
                a     = base_args(recon, L);
                first = false;
            }
            DlfPlaneJob &J = a.job[a.njob];
            J              = plane_job(s, recon, plane, true);
            J.src          = recon->plane[plane];
            J.src_stride   = recon->stride[plane];
            J.ref          = src->plane[plane];
            J.ref_stride   = src->stride[plane];
            J.ntrial       = mi;
            for (int k = 0; k < mi; k++) { // the trial's tables of this plane only (try_filter_frame's levels)
                SvtGpuLfParams q = p;
                set_trial_level(q, plane, srch[i]->dir, lv[i][k]);
                const int  base[3][2] = {{q.filter_level[0], q.filter_level[1]},
                                         {q.filter_level_u, q.filter_level_u},
                                         {q.filter_level_v, q.filter_level_v}};
                const bool on = plane_active(q, plane);
                for (int dir = 0; dir < 2; dir++) {
                    if (on) fill_level_table(q, plane, dir, base[plane][dir], J.lvl[k][dir]);
                    else std::memset(J.lvl[k][dir], 0, 128);
                }
            }
            m[a.njob]   = mi;
            who[a.njob] = i;
            a.njob++;
        }
        if (first) return SVTGPU_OK; // every search has finished
        a.sse    = s->d_sse;
        a.arrive = s->d_arrive;
        a.out    = s->h_sse_dev;
        a.seq    = ++s->seq;
        if (int rc = launch_tile(a, recon->bytes_per_sample, true, st)) return rc;
        if (int rc = svtgpu_wait_seq(s->h_sse + MAX_JOBS * MAX_TRIALS, a.seq, st)) return rc;
        svtgpu_count_xfer(1, 8); // the sequence word
        unsigned long long sse[MAX_JOBS * MAX_TRIALS];
        std::memcpy(sse, s->h_sse, sizeof sse);
        for (int j = 0; j < a.njob; j++) svtgpu_count_xfer(1, 8 * (size_t)m[j]); // the job's trial SSEs (mapped memory)
        // a picture tiled over GPUs: every rank measured its tile; the frame's SSE is the sum over the ranks, and
        // every rank then takes the same bisection step
        if (int rc = svtgpu_comm_sum(s->comm, sse, MAX_JOBS * MAX_TRIALS, false, st, SVTGPU_XCH_DLF)) return rc;
        for (int j = 0; j < a.njob; j++) srch[who[j]]->feed(lv[who[j]], m[j], sse + j * MAX_TRIALS);
    }
}

bool valid_params(const SvtGpuLfParams *p) {
    if (!p) return false;
    const int lv[4] = {p->filter_level[0], p->filter_level[1], p->filter_level_u, p->filter_level_v};
    for (int v : lv)
        if (v < 0 || v > 63) return false;
    return p->sharpness_level >= 0 && p->sharpness_level <= 7;
}

} // namespace

extern "C" int svtgpu_dlf_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuDlfState **out) {
    if (!ctx || !out || width <= 0 || height <= 0 || (width & 7) || (height & 7)) return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    SvtGpuDlfState *s = new SvtGpuDlfState();
    s->ctx     = ctx;
    s->width   = width;
    s->height  = height;
    s->mi_cols = width >> 2;
    s->mi_rows = height >> 2;
    s->crop_w  = width, s->crop_h = height;
    s->uw[0]   = width / 4, s->uh[0] = height / 4;
    s->uw[1]   = width / 8, s->uh[1] = height / 8;
    s->sse_rect[2] = s->out_rect[2] = width, s->sse_rect[3] = s->out_rect[3] = height;
    hipError_t e = hipMalloc(&s->d_mi, sizeof(SvtGpuLfMi) * s->mi_rows * s->mi_cols);
    for (int c = 0; c < 2 && e == hipSuccess; c++)
        for (int d = 0; d < 2 && e == hipSuccess; d++)
            e = hipMalloc(&s->d_rec[c][d], sizeof(uint32_t) * s->uw[c] * s->uh[c]);
    if (e == hipSuccess) // the three planes' copies for an in-place apply
        e = hipMalloc(&s->d_scratch, ((size_t)width * height + 2 * (size_t)((width + 1) >> 1) * ((height + 1) >> 1)) * 2);
    if (e == hipSuccess) e = hipMalloc(&s->d_sse, sizeof(unsigned long long) * MAX_JOBS * MAX_TRIALS);
    if (e == hipSuccess) e = hipMalloc(&s->d_arrive, sizeof(unsigned int));
    if (e == hipSuccess) e = hipMemset(s->d_sse, 0, sizeof(unsigned long long) * MAX_JOBS * MAX_TRIALS);
    if (e == hipSuccess) e = hipMemset(s->d_arrive, 0, sizeof(unsigned int));
    if (e == hipSuccess)
        e = hipHostMalloc(&s->h_sse, sizeof(unsigned long long) * (MAX_JOBS * MAX_TRIALS + 2),
                          hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) s->h_sse[MAX_JOBS * MAX_TRIALS] = s->h_sse[MAX_JOBS * MAX_TRIALS + 1] = 0;
    if (e == hipSuccess) e = hipHostGetDevicePointer((void **)&s->h_sse_dev, s->h_sse, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        svtgpu_dlf_state_destroy(s);
        svtgpu_set_last_hip_error(e, "dlf state alloc", __FILE__, __LINE__);
        return e == hipErrorOutOfMemory ? SVTGPU_ERR_OOM : SVTGPU_ERR_HIP;
    }
    *out = s;
    return SVTGPU_OK;
}

extern "C" void svtgpu_dlf_state_destroy(SvtGpuDlfState *s) {
    if (!s) return;
    (void)hipFree(s->d_mi);
    if (s->h_mi) (void)hipHostFree(s->h_mi);
    if (s->mi_free) (void)hipEventDestroy(s->mi_free);
    for (int c = 0; c < 2; c++)
        for (int d = 0; d < 2; d++) (void)hipFree(s->d_rec[c][d]);
    (void)hipFree(s->d_scratch);
    (void)hipFree(s->d_sse);
    (void)hipFree(s->d_arrive);
    if (s->h_sse) (void)hipHostFree(s->h_sse);
    (void)hipFree(s->d_search);
    (void)hipFree(s->d_plans);
    (void)hipFree(s->d_res);
    if (s->h_res) (void)hipHostFree(s->h_res);
    svtgpu_prio_destroy(&s->prio);
    if (s->h_search) (void)hipHostFree(s->h_search);
    delete s;
}

namespace {
// the edge records of both plane types and directions from s->d_mi; `bad` (device-side checks) or null
int edge_records(SvtGpuDlfState *s, hipStream_t st, unsigned long long *bad) {
    for (int c = 0; c < 2; c++)
        for (int d = 0; d < 2; d++) {
            hipLaunchKernelGGL(dlf_edge_records_kernel, dim3((s->uw[c] + 127) / 128, s->uh[c]), dim3(128), 0, st,
                               s->d_mi, s->mi_cols, s->uw[c], s->uh[c], c, d == 0, s->crop_w >> c, s->crop_h >> c,
                               s->d_rec[c][d], bad);
            HIP_TRY(hipGetLastError());
        }
    s->have_mi = 1;
    return SVTGPU_OK;
}

// a device-side check raised the flag: the grid handed over had records out of range (cleared when reported)
bool take_bad_mi(SvtGpuDlfState *s) {
    volatile unsigned long long *f = s->h_sse + MAX_JOBS * MAX_TRIALS + 1;
    if (!*f) return false;
    *f = 0;
    return true;
}
} // namespace

extern "C" int svtgpu_dlf_set_crop(SvtGpuDlfState *s, int32_t crop_width, int32_t crop_height) {
    if (!s || crop_width <= s->width - 8 || crop_width > s->width || crop_height <= s->height - 8 ||
        crop_height > s->height)
        return SVTGPU_ERR_INVALID_ARG; // the coded size is the crop rounded up to 8
    // the edge records stop at the crop: records built for another crop are stale, so filter / pick refuse until the
    // next svtgpu_dlf_set_mode_info(_device) rebuilds them
    if (crop_width != s->crop_w || crop_height != s->crop_h) s->have_mi = 0;
    s->crop_w = crop_width, s->crop_h = crop_height;
    return SVTGPU_OK;
}

extern "C" int svtgpu_dlf_set_mode_info(SvtGpuDlfState *s, const SvtGpuLfMi *mi, void *stream) {
    if (!s || !mi) return SVTGPU_ERR_INVALID_ARG;
    const size_t n = (size_t)s->mi_rows * s->mi_cols;
    for (size_t i = 0; i < n; i++) { // the device tables are indexed by these fields
        const SvtGpuLfMi &m = mi[i];
        if (m.bsize >= kNumBsize || m.tx_depth > 2 || m.ref_frame0 < 0 || m.ref_frame0 > 7 || m.mode > 24 ||
            m.segment_id > 7)
            return SVTGPU_ERR_INVALID_ARG;
    }
    hipStream_t st = pick_stream(s->ctx, stream);
    // the caller's grid goes through pinned staging, so the upload is asynchronous and the caller may reuse its
    // buffer at once (an encoder hands over a new grid every frame)
    if (!s->h_mi) {
        HIP_TRY(hipHostMalloc((void **)&s->h_mi, n * sizeof(SvtGpuLfMi), hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&s->mi_free, hipEventDisableTiming));
    } else {
        HIP_TRY(hipEventSynchronize(s->mi_free)); // the previous frame's upload has read the staging
    }
    std::memcpy(s->h_mi, mi, n * sizeof(SvtGpuLfMi));
    HIP_TRY(hipMemcpyAsync(s->d_mi, s->h_mi, n * sizeof(SvtGpuLfMi), hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(s->mi_free, st));
    svtgpu_count_xfer(0, n * sizeof(SvtGpuLfMi));
    s->mi_on_device = 0;
    return edge_records(s, st, nullptr);
}

extern "C" int svtgpu_dlf_set_mode_info_device(SvtGpuDlfState *s, const SvtGpuLfMi *d_mi, void *stream) {
    if (!s || !d_mi) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    // a grid already in HBM (an encoder whose mode decision runs on the device): one copy in stream order, checked
    // by the records kernel itself -- no host pass over the records, no PCIe
    HIP_TRY(hipMemcpyAsync(s->d_mi, d_mi, (size_t)s->mi_rows * s->mi_cols * sizeof(SvtGpuLfMi),
                           hipMemcpyDeviceToDevice, st));
    // this grid's verdict only: the flag word (mapped memory) is cleared in stream order before its records kernel
    HIP_TRY(hipMemsetAsync(s->h_sse_dev + MAX_JOBS * MAX_TRIALS + 1, 0, sizeof(unsigned long long), st));
    s->mi_on_device = 1;
    return edge_records(s, st, s->h_sse_dev + MAX_JOBS * MAX_TRIALS + 1);
}

extern "C" int svtgpu_dlf_set_tile(SvtGpuDlfState *s, const int32_t sse_rect[4], const int32_t out_rect[4],
                                   SvtGpuComm *comm) {
    if (!s) return SVTGPU_ERR_INVALID_ARG;
    const int32_t whole[4] = {0, 0, s->width, s->height};
    const int32_t *r[2]    = {sse_rect ? sse_rect : whole, out_rect ? out_rect : whole};
    for (const int32_t *q : r) // 8-aligned (chroma 4-aligned: the tile staging reads aligned 4-sample groups)
        if (q[0] < 0 || q[1] < 0 || q[2] > s->width || q[3] > s->height || q[0] >= q[2] || q[1] >= q[3] ||
            ((q[0] | q[1]) & 7) || ((q[2] & 7) && q[2] != s->width) || ((q[3] & 7) && q[3] != s->height))
            return SVTGPU_ERR_INVALID_ARG;
    std::memcpy(s->sse_rect, r[0], sizeof s->sse_rect);
    std::memcpy(s->out_rect, r[1], sizeof s->out_rect);
    s->comm = comm;
    return SVTGPU_OK;
}

namespace {
// filter planes [ps, pe) of `in` into `out`, the filtered planes in one launch (one job per plane); in == out is
// allowed (the planes are staged in scratch)
int dlf_frame_impl(SvtGpuDlfState *s, const SvtGpuFrame *in, SvtGpuFrame *out, const SvtGpuLfParams *params,
                   int32_t ps, int32_t pe, hipStream_t st) {
    // params == nullptr: the levels of the last svtgpu_dlf_pick_async, as level tables on the device (every plane goes
    // through the tile kernel: a plane that is not filtered has all-zero tables, lists no edge and is copied)
    const bool dev = params == nullptr;
    if (dev) params = &s->dev_params;
    if (s->mi_on_device && !dev) { // a device grid no pick has reported on (the FROM_Q levels): its verdict first
        s->mi_on_device = 0;
        if (int rc = svtgpu_comm_wait(s->comm, st)) return rc; // bounded when an exchange may sit before it
        if (take_bad_mi(s)) return SVTGPU_ERR_INVALID_ARG;
    }
    LevelTables L;
    build_level_tables(*params, L);
    bool        luma_off = false;
    DlfTileArgs a        = base_args(in, L);
    size_t      sc_off   = 0; // bytes of scratch used by earlier planes
    for (int pl = ps; pl < pe; pl++) {
        if (pl == 0 && !plane_active(*params, 0)) luma_off = true; // no plane is filtered (:575-577)
        const size_t bps = in->bytes_per_sample;
        const bool   on  = dev || (!luma_off && plane_active(*params, pl));
        if (!on) { // the output rectangle of the plane passes through
            const DlfPlaneJob R = plane_job(s, in, pl, false);
            if (in != out && R.ow > 0 && R.oh > 0) {
                const size_t io = ((size_t)R.oy * in->stride[pl] + R.ox) * bps, oo = ((size_t)R.oy * out->stride[pl] + R.ox) * bps;
                HIP_TRY(hipMemcpy2DAsync((uint8_t *)out->plane[pl] + oo, out->stride[pl] * bps,
                                         (const uint8_t *)in->plane[pl] + io, in->stride[pl] * bps, R.ow * bps, R.oh,
                                         hipMemcpyDeviceToDevice, st));
            }
            continue;
        }
        DlfPlaneJob &J = a.job[a.njob];
        J              = plane_job(s, in, pl, false);
        if (!J.tiles) continue;
        a.njob++;
        if (in == out) {
            void *sc = (uint8_t *)s->d_scratch + sc_off;
            sc_off += (size_t)in->pw[pl] * in->ph[pl] * bps;
            HIP_TRY(hipMemcpy2DAsync(sc, in->pw[pl] * bps, in->plane[pl], in->stride[pl] * bps,
                                     in->pw[pl] * bps, in->ph[pl], hipMemcpyDeviceToDevice, st));
            J.src        = sc;
            J.src_stride = in->pw[pl];
        } else {
            J.src        = in->plane[pl];
            J.src_stride = in->stride[pl];
        }
        J.dst        = out->plane[pl];
        J.dst_stride = out->stride[pl];
        J.ntrial     = 1;
        for (int dir = 0; dir < 2; dir++) std::memcpy(J.lvl[0][dir], L.lvl[pl][dir], 128);
    }
    if (dev) a.dev_lvl = ((const DlfDevResult *)s->d_res)->lvl[0][0];
    if (a.njob) return launch_tile(a, (int)in->bytes_per_sample, false, st);
    return SVTGPU_OK;
}
} // namespace

extern "C" int svtgpu_dlf_frame(SvtGpuDlfState *s, SvtGpuFrame *frame, const SvtGpuLfParams *params,
                                int32_t plane_start, int32_t plane_end, void *stream) {
    if (!s || !frame_matches(s, frame) || (params ? !valid_params(params) : !s->dev_ready) || plane_start < 0 || plane_end > 3 ||
        plane_start > plane_end || !s->have_mi)
        return SVTGPU_ERR_INVALID_ARG;
    return dlf_frame_impl(s, frame, frame, params, plane_start, plane_end, pick_stream(s->ctx, stream));
}

extern "C" int svtgpu_dlf_frame_to(SvtGpuDlfState *s, const SvtGpuFrame *in, SvtGpuFrame *out,
                                   const SvtGpuLfParams *params, int32_t plane_start, int32_t plane_end,
                                   void *stream) {
    if (!s || !frame_matches(s, in) || !frame_matches(s, out) || in->bit_depth != out->bit_depth ||
        (params ? !valid_params(params) : !s->dev_ready) || plane_start < 0 || plane_end > 3 || plane_start > plane_end ||
        !s->have_mi)
        return SVTGPU_ERR_INVALID_ARG;
    return dlf_frame_impl(s, in, out, params, plane_start, plane_end, pick_stream(s->ctx, stream));
}

extern "C" int svtgpu_dlf_pick(SvtGpuDlfState *s, SvtGpuFrame *recon, const SvtGpuFrame *source,
                               SvtGpuLfParams *params, int32_t dlf_avg, int32_t dlf_avg_uv,
                               int32_t temporal_layer_index, int32_t early_exit_convergence,
                               int32_t tx_mode_only_4x4, void *stream) {
    if (!s || !frame_matches(s, recon) || !frame_matches(s, source) || source->bit_depth != recon->bit_depth ||
        !valid_params(params) || !s->have_mi)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t    st = pick_stream(s->ctx, stream);
    SvtGpuLfParams p  = *params;
    p.sharpness_level = 0;
    const int last[4] = {p.filter_level[0], p.filter_level[1], p.filter_level_u, p.filter_level_v};
    int       rc;
    // The three searches are independent: a trial filters only its own plane with its own level (the luma levels
    // gate only the luma plane, EbDeblockingFilter.c:571-577), so they share launches.  With dlf_avg_uv on a
    // non-base layer the chroma levels stay (EbDeblockingFilter.c:1221-1229).
    const bool  search_uv = !(dlf_avg_uv && temporal_layer_index > 0);
    LevelSearch ys(last, dlf_avg, early_exit_convergence, tx_mode_only_4x4, 0, 2);
    LevelSearch us(last, dlf_avg, early_exit_convergence, tx_mode_only_4x4, 1, 0);
    LevelSearch vs(last, dlf_avg, early_exit_convergence, tx_mode_only_4x4, 2, 0);
    LevelSearch *all[3] = {&ys, &us, &vs};
    const int   chunk  = dlf_device_chunk(s);
    hipStream_t hs;
    if ((rc = svtgpu_prio_enter(&s->prio, st, &hs))) return rc;
    rc = chunk ? run_searches_device(s, recon, source, p, all, search_uv ? 3 : 1, hs, chunk)
               : run_searches(s, recon, source, p, all, search_uv ? 3 : 1, hs);
    if (int rj = svtgpu_prio_leave(&s->prio, hs, st)) rc = rc ? rc : rj;
    if (rc) return rc;
    if (s->mi_on_device) { // the grid was checked by the records kernel: its verdict, once the stream has passed it
        s->mi_on_device = 0;
        if (int rc = svtgpu_comm_wait(s->comm, st)) return rc;
        if (take_bad_mi(s)) return SVTGPU_ERR_INVALID_ARG;
    }
    p.filter_level[0] = p.filter_level[1] = ys.best;
    p.filter_level_u = search_uv ? us.best : last[2];
    p.filter_level_v = search_uv ? vs.best : last[3];
    *params          = p;
    return SVTGPU_OK;
}

// The level search with no host wait: the start (dlf_search_init_kernel), a number of device trial rounds sized from the
// previous search's count, each stepping itself (dlf_trial_dev_kernel), then dlf_finish_kernel, which completes a search
// still open and writes the apply's tables and the caller's levels -- all in stream order.  A picture tiled over GPUs
// (an all-reduce between a trial round and its step) runs the synchronous search here and keeps its levels.
extern "C" int svtgpu_dlf_pick_async(SvtGpuDlfState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                     const SvtGpuLfParams *params, int32_t dlf_avg, int32_t dlf_avg_uv,
                                     int32_t temporal_layer_index, int32_t early_exit_convergence,
                                     int32_t tx_mode_only_4x4, void *stream) {
    if (!s || !frame_matches(s, recon) || !frame_matches(s, source) || source->bit_depth != recon->bit_depth ||
        !valid_params(params) || !s->have_mi)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    if (!s->d_res) {
        HIP_TRY(hipMalloc(&s->d_res, sizeof(DlfDevResult)));
        HIP_TRY(hipHostMalloc(&s->h_res, sizeof(DlfDevResult), hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(s->h_res, 0, sizeof(DlfDevResult));
        HIP_TRY(hipHostGetDevicePointer(&s->h_res_dev, s->h_res, 0));
    }
    if (svtgpu_comm_tiled(s->comm)) { // the tiled search (host read-backs per chunk); its levels become the result
        SvtGpuLfParams p = *params;
        if (int rc = svtgpu_dlf_pick(s, const_cast<SvtGpuFrame *>(recon), source, &p, dlf_avg, dlf_avg_uv, temporal_layer_index,
                                     early_exit_convergence, tx_mode_only_4x4, stream))
            return rc;
        DlfDevResult r;
        std::memset(&r, 0, sizeof r);
        LevelTables L;
        build_level_tables(p, L);
        const bool luma_off = !plane_active(p, 0);
        for (int pl = 0; pl < 3; pl++)
            if (!luma_off && plane_active(p, pl)) std::memcpy(r.lvl[pl], L.lvl[pl], sizeof r.lvl[pl]);
        r.levels[0] = p.filter_level[0], r.levels[1] = p.filter_level[1], r.levels[2] = p.filter_level_u;
        r.levels[3] = p.filter_level_v, r.seq = ++s->dev_seq;
        std::memcpy(s->h_res, &r, sizeof r);
        HIP_TRY(hipMemcpyAsync(s->d_res, s->h_res, sizeof r, hipMemcpyHostToDevice, st));
        s->dev_params = p, s->dev_ready = 1, s->dev_pending = 1;
        return SVTGPU_OK;
    }
    if (!s->d_search) {
        HIP_TRY(hipMalloc(&s->d_search, sizeof(DlfDevSearch)));
        HIP_TRY(hipHostMalloc(&s->h_search, sizeof(DlfDevSearch), hipHostMallocDefault));
    }
    if (!s->d_plans) HIP_TRY(hipMalloc(&s->d_plans, 2 * sizeof(DlfDevPlan)));
    // the rounds to enqueue: one more than the previous search took (read from mapped memory without waiting: the
    // previous result when it is already there, else the last hint); SVTGPU_DLF_ROUNDS=k fixes it (tests: 1 makes the
    // finish kernel complete the search)
    static const int fixed = [] {
        const char *e = std::getenv("SVTGPU_DLF_ROUNDS");
        return e ? std::max(1, std::min(64, std::atoi(e))) : 0;
    }();
    // the latest search that has completed (whichever: the caller's thread may run ahead of the device) sizes the next
    // one's rounds with a margin of two
    const volatile DlfDevResult *hr = (const volatile DlfDevResult *)s->h_res;
    if (hr->seq != s->dev_seen) s->dev_seen = hr->seq, s->dev_rounds = std::max(4, std::min(16, hr->rounds + 2));
    const int rounds = fixed ? fixed : s->dev_rounds;
    s->dev_rounds_last = rounds;
    SvtGpuLfParams p  = *params;
    p.sharpness_level = 0;
    const int ns      = (dlf_avg_uv && temporal_layer_index > 0) ? 1 : 3;
    DlfDevSearch *D   = (DlfDevSearch *)s->d_search;
    hipLaunchKernelGGL(dlf_search_init_kernel, dim3(1), dim3(64), 0, st, D, p, ns, dlf_avg, early_exit_convergence,
                       tx_mode_only_4x4);
    HIP_TRY(hipGetLastError());
    DlfDevPlan *plans = (DlfDevPlan *)s->d_plans; // trial launch k reads plans[k & 1] and its step writes the other
    HIP_TRY(hipMemcpyAsync(&plans[0], &D->plan, sizeof(DlfDevPlan), hipMemcpyDeviceToDevice, st));
    LevelTables L;
    build_level_tables(p, L); // the thresholds (sharpness 0); the levels come from the plan
    DlfTileArgs a = base_args(recon, L);
    int         max_items = 0;
    for (int i = 0; i < ns; i++) {
        DlfPlaneJob &J = a.job[i];
        J              = plane_job(s, recon, i, true);
        J.src = recon->plane[i], J.src_stride = recon->stride[i];
        J.ref = source->plane[i], J.ref_stride = source->stride[i];
        J.ntrial = MAX_TRIALS;
        max_items += J.tiles * MAX_TRIALS;
    }
    a.njob = ns, a.sse = s->d_sse, a.arrive = s->d_arrive, a.plan = &D->plan, a.dyn = 1;
    const int grid = std::max(1, max_items);
    for (int k = 0; k < rounds; k++) {
        a.plan = &plans[k & 1], a.next_plan = &plans[(k + 1) & 1];
        if (recon->bytes_per_sample == 2)
            hipLaunchKernelGGL(dlf_trial_dev_kernel<uint16_t>, dim3(grid), dim3(NTHR), 0, st, a, D, 1);
        else
            hipLaunchKernelGGL(dlf_trial_dev_kernel<uint8_t>, dim3(grid), dim3(NTHR), 0, st, a, D, 1);
        HIP_TRY(hipGetLastError());
    }
    a.plan = &D->plan, a.next_plan = nullptr; // the finisher: one workgroup stepping the search's own copy
    const int seq = ++s->dev_seq;
    if (recon->bytes_per_sample == 2)
        hipLaunchKernelGGL(dlf_finish_kernel<uint16_t>, dim3(1), dim3(NTHR), 0, st, a, D, (DlfDevResult *)s->d_res,
                           (DlfDevResult *)s->h_res_dev, seq);
    else
        hipLaunchKernelGGL(dlf_finish_kernel<uint8_t>, dim3(1), dim3(NTHR), 0, st, a, D, (DlfDevResult *)s->d_res,
                           (DlfDevResult *)s->h_res_dev, seq);
    HIP_TRY(hipGetLastError());
    s->dev_params = p, s->dev_ready = 1, s->dev_pending = 1;
    return SVTGPU_OK;
}

extern "C" int svtgpu_dlf_read_levels(SvtGpuDlfState *s, SvtGpuLfParams *params_out, void *stream) {
    if (!s || !params_out || !s->dev_ready) return SVTGPU_ERR_INVALID_ARG;
    if (s->dev_pending) {
        if (int rc = svtgpu_comm_wait(s->comm, pick_stream(s->ctx, stream))) return rc;
        s->dev_pending = 0;
        if (((const volatile DlfDevResult *)s->h_res)->seq != s->dev_seq) {
            svtgpu_set_last_hip_error(hipErrorUnknown, "dlf asynchronous level search: result word missing after the "
                                      "stream wait", __FILE__, __LINE__);
            return SVTGPU_ERR_HIP;
        }
        if (s->mi_on_device) { // the device grid's verdict (its records kernel ran before the search)
            s->mi_on_device = 0;
            if (take_bad_mi(s)) return SVTGPU_ERR_INVALID_ARG;
        }
    }
    const volatile DlfDevResult *r = (const volatile DlfDevResult *)s->h_res;
    SvtGpuLfParams               p = s->dev_params;
    p.filter_level[0] = r->levels[0], p.filter_level[1] = r->levels[1];
    p.filter_level_u = r->levels[2], p.filter_level_v = r->levels[3];
    *params_out = p;
    return SVTGPU_OK;
}

extern "C" int svtgpu_dlf_async_rounds(const SvtGpuDlfState *s, int32_t *taken, int32_t *enqueued) {
    if (!s || !s->h_res) return SVTGPU_ERR_INVALID_ARG;
    if (taken) *taken = ((const volatile DlfDevResult *)s->h_res)->rounds;
    if (enqueued) *enqueued = s->dev_rounds_last;
    return SVTGPU_OK;
}

extern "C" int svtgpu_plane_sse(const SvtGpuFrame *a, const SvtGpuFrame *b, int32_t plane, uint64_t *sse,
                                void *stream) {
    if (!a || !b || !sse || plane < 0 || plane > 2 || a->width != b->width || a->height != b->height ||
        a->bytes_per_sample != b->bytes_per_sample)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(a->ctx, stream);
    static thread_local unsigned long long *d = nullptr; // per-thread result slot
    if (!d) HIP_TRY(hipMalloc((void **)&d, sizeof *d));
    HIP_TRY(hipMemsetAsync(d, 0, sizeof *d, st));
    const int rows = a->ph[plane], blocks = std::min(rows, 1024);
    if (a->bytes_per_sample == 2)
        hipLaunchKernelGGL(plane_sse_kernel<uint16_t>, dim3(blocks), dim3(256), 0, st, (const uint16_t *)a->plane[plane],
                           a->stride[plane], (const uint16_t *)b->plane[plane], b->stride[plane], a->pw[plane], rows, d);
    else
        hipLaunchKernelGGL(plane_sse_kernel<uint8_t>, dim3(blocks), dim3(256), 0, st, (const uint8_t *)a->plane[plane],
                           a->stride[plane], (const uint8_t *)b->plane[plane], b->stride[plane], a->pw[plane], rows, d);
    HIP_TRY(hipGetLastError());
    unsigned long long h = 0;
    HIP_TRY(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *sse = h;
    return SVTGPU_OK;
}

// ---------------------------------------------------------------------------------------------
// RTCD-compatible per-segment shims (common_dsp_rtcd.h:1115-1146): synchronous, for unit parity
// ---------------------------------------------------------------------------------------------
namespace {
template <typename T>
void lpf_shim(T *s, int32_t pitch, int vertical, int len, const uint8_t *blimit, const uint8_t *limit,
              const uint8_t *thresh, int bd) {
    const long step = vertical ? 1 : pitch, adv = vertical ? pitch : 1;
    const int  h    = len == 14 ? 7 : len == 8 ? 4 : len == 6 ? 3 : 2;
    uint16_t   lines[4 * 16] = {0};
    for (int l = 0; l < 4; l++) // only the samples the reference function touches
        for (int k = -h; k < h; k++) lines[l * 16 + 8 + k] = s[l * adv + k * step];
    hipStream_t st = svtgpu_shim_stream();
    static thread_local uint16_t *d = nullptr;
    if (!d) HIP_OR_DIE(hipMalloc(&d, sizeof lines));
    HIP_OR_DIE(hipMemcpyAsync(d, lines, sizeof lines, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(lpf_lines_kernel, dim3(1), dim3(64), 0, st, d, len, (int)*blimit, (int)*limit, (int)*thresh, bd);
    HIP_OR_DIE(hipGetLastError());
    HIP_OR_DIE(hipMemcpyAsync(lines, d, sizeof lines, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int l = 0; l < 4; l++)
        for (int k = -h; k < h; k++) s[l * adv + k * step] = (T)lines[l * 16 + 8 + k];
}
} // namespace

#define LPF_SHIMS(DIR, VERT, N)                                                                           \
    extern "C" void svtgpu_lpf_##DIR##_##N(uint8_t *s, int32_t pitch, const uint8_t *blimit,               \
                                           const uint8_t *limit, const uint8_t *thresh) {                  \
        lpf_shim<uint8_t>(s, pitch, VERT, N, blimit, limit, thresh, 8);                                    \
    }                                                                                                      \
    extern "C" void svtgpu_highbd_lpf_##DIR##_##N(uint16_t *s, int32_t pitch, const uint8_t *blimit,       \
                                                  const uint8_t *limit, const uint8_t *thresh, int32_t bd) { \
        lpf_shim<uint16_t>(s, pitch, VERT, N, blimit, limit, thresh, bd);                                  \
    }
LPF_SHIMS(horizontal, 0, 4)
LPF_SHIMS(horizontal, 0, 6)
LPF_SHIMS(horizontal, 0, 8)
LPF_SHIMS(horizontal, 0, 14)
LPF_SHIMS(vertical, 1, 4)
LPF_SHIMS(vertical, 1, 6)
LPF_SHIMS(vertical, 1, 8)
LPF_SHIMS(vertical, 1, 14)
