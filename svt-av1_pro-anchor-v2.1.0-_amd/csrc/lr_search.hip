// lr_search.hip — loop-restoration parameter search on gfx950 (restoration_seg_search + rest_finish_search).
//
// Reference: Source/Lib/Encoder/Codec/EbRestorationPick.c (search :129-1460, finish :1555-1634), with the filters
// of Common/Codec/EbRestoration.c and convolve.c; the rate helpers of EbEntropyCoding.c:2876-3022.
//
// The search runs without stripe boundaries (use_boundaries_in_rest_search = 0, EbEncHandle.c:4162), so every
// filter output is a per-pixel function of the edge-clamped CDEF output.  All searched planes are processed
// together over one tile list (<= 64x64 tiles aligned to each restoration unit, planes in order):
//   unit_sums_kernel      Σ dgd (Wiener average) and the RESTORE_NONE SSE per unit
//   wiener_stats_kernel   the 7x7 (5x5, 3x3) Wiener statistics M, H of svt_av1_compute_stats: a lane group per
//                         window-column pair accumulates its 7x7 block with v_dot2_i32_i16 over horizontal pixel
//                         pairs (diagonal groups also form M); per-tile partials are reduced per unit
//   sgr_flt_kernel        box sums of a tile once, then for every searched ep the A/B maps and both self-guided
//                         filters (kept in HBM as int16)
//   wiener_solve_kernel   the int64 fixed-point Wiener decomposition and score per unit (the descent's seed)
//   wiener_res_kernel     the whole Wiener descent of finer_tile_search_wiener_seg per unit with the unit resident on
//                         the CU: CDEF window in LDS, source in registers, a rolling horizontal pass per lane; units
//                         too large for one CU are cut into row parts whose SSEs meet each candidate
//   sgr_res_kernel        the whole self-guided search of one (unit, ep) with the unit resident on the CU: the
//                         ep's filter planes read once into registers, the projection moments, the seed (the 2x2
//                         double solve, as the reference) and finer_search_pixel_proj_error's descent, stepped by a
//                         control wave between passes over the resident pixels
//   sgr_best_kernel, sgr_sse_kernel
//                         best ep per unit (strict <) and the SSE of its clipped output
// The host does what is sequential in the reference and cheap: the RD pass over the units (rest_finish_search).  A
// frame costs one host wait (the final read-back).
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include "lr_common.h"


namespace {

struct Tile {
    int32_t plane, unit, x0, y0, w, h; // unit: global index over the searched planes
};
struct URect {
    int32_t h_start, h_end, v_start, v_end;
};
constexpr int PRJ_MIN0 = -96, PRJ_MAX0 = 31, PRJ_MIN1 = -32, PRJ_MAX1 = 95;
const int     kHostSgrR[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                              {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};
// r = 1 s values of the sets (c_sgr_s[.][1]): eps 2/11, 5/12 and 8/13 share theirs, so their r = 1 filters are equal
const int     kHostSgrS1[16] = {3236, 2158, 1618, 1438, 1295, 1177, 1079, 996, 925, 863, 2589, 1618, 1177, 925, -1, -1};

struct PlaneArgs {
    const void *dgd, *src;
    int16_t    *flt; // [ne][2][H][fstride] self-guided outputs minus the scaled source, g = flt - (dgd << 4) (int16)
    int16_t    *dxp; // [H][fstride] dgd - src (int16; planes with a self-guided search, else null)
    int32_t     dstride, sstride, W, H, bd, fstride;
    int32_t     unit_base, pair_base, ne; // SGR pair of (unit, k) = pair_base + (unit - unit_base) * ne + k
    int32_t     eps[16];
    int32_t     f1e[16];                  // the ep slot whose r = 1 plane holds slot k's (equal s: same filter)
    int32_t     win, nval;                // Wiener window and statistics values per unit
    int64_t     mh_off;                   // this plane's statistics in the M/H buffer (int64 elements)
};
struct SearchArgs {
    PlaneArgs      pl[3];
    const Tile    *tiles;
    const URect   *units;
    const int32_t *tile0; // first tile of every global unit, plus the end
};

template <typename T>
__device__ inline int px(const T *p, int stride, int W, int H, int y, int x) {
    y = min(max(y, 0), H - 1);
    x = min(max(x, 0), W - 1);
    return p[(size_t)y * stride + x];
}

// wave total in lane 63 (svtgpu_internal.h)
__device__ inline unsigned long long wave_sum(unsigned long long v) { return wave_sum_lane63(v); }
constexpr int WAVE_LAST = 63;

// Kernel timing for svtgpu_lr_profile: with a slot `tk`, the earliest workgroup start (atomicMin) and the latest
// workgroup end (atomicMax, at tk + PROF_NL * PROF_SP) of a launch on the 100 MHz s_memrealtime clock, spread over
// PROF_SP addresses by workgroup index so that thousands of workgroups do not contend on one line -- the launch's
// device duration without per-launch event packets (which cost far more than these launches).
constexpr int PROF_NL = 512, PROF_SP = 64;
#define PROF_BEGIN(tk)                                                                                      \
    if ((tk) && threadIdx.x == 0)                                                                           \
    atomicMin((tk) + (blockIdx.x & (PROF_SP - 1)), (unsigned long long)__builtin_amdgcn_s_memrealtime())
#define PROF_END(tk)                                                                                        \
    if (tk) {                                                                                               \
        __syncthreads();                                                                                    \
        if (threadIdx.x == 0)                                                                               \
            atomicMax((tk) + PROF_NL * PROF_SP + (blockIdx.x & (PROF_SP - 1)),                              \
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());                                \
    }

typedef short v2i16 __attribute__((ext_vector_type(2)));
__device__ inline int dot2(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16, a), __builtin_bit_cast(v2i16, b), c, false);
}
// clamp of a lane value to [0, hi] (hi wave-uniform) in one instruction (the compiler emits a max and a min)
__device__ inline int clamp0_s(int v, int hi_uniform) {
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "s"(hi_uniform));
    return r;
}
// the same with a wave-uniform accumulator input held in an SGPR: the VOP3P form, where the compiler would copy a
// constant into the destination of an accumulating v_dot2c for every call
__device__ inline int dot2_s(uint32_t a, uint32_t b, int c_uniform) {
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c_uniform));
    return r;
}

template <typename T>
__device__ inline void load4(const T *p, int *v) {
    if constexpr (sizeof(T) == 2) {
        const uint2 w = *(const uint2 *)p;
        v[0] = w.x & 0xFFFF, v[1] = w.x >> 16, v[2] = w.y & 0xFFFF, v[3] = w.y >> 16;
    } else {
        const uint32_t w = *(const uint32_t *)p;
        v[0] = w & 0xFF, v[1] = (w >> 8) & 0xFF, v[2] = (w >> 16) & 0xFF, v[3] = w >> 24;
    }
}
__device__ inline void load4s(const int16_t *p, int *v) {
    const int2 w = *(const int2 *)p;
    v[0] = (int)(int16_t)(w.x & 0xFFFF), v[1] = w.x >> 16, v[2] = (int)(int16_t)(w.y & 0xFFFF), v[3] = w.y >> 16;
}

// the low halves of lo and hi as one packed int16 pair: one v_perm_b32 (the and + shift-or form took two VALU ops)
__device__ inline uint32_t pack2(int lo, int hi) { return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u); }

// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void unit_sums_kernel(const SearchArgs A, unsigned long long *sum,
                                                        unsigned long long *sse, unsigned long long *tk) {
    PROF_BEGIN(tk);
    const Tile       t = A.tiles[xcd_swizzle(blockIdx.x, gridDim.x)];
    const PlaneArgs &P = A.pl[t.plane];
    const T         *d = (const T *)P.dgd, *s = (const T *)P.src;
    uint32_t ps = 0, pe = 0; // <= 16 samples per lane: fits 32 bits
    // 4-sample chunks (tile x offsets are multiples of 4): chunk k of this lane is row (threadIdx.x >> 4) + 16 k,
    // columns 4 (threadIdx.x & 15) .. + 3; all four chunks' loads are issued first.  A plane whose crop width is not a
    // multiple of 4 ends in a partial chunk: its samples past the crop are read one by one and left out
    int dv[4][4], sv[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int r = (threadIdx.x >> 4) + 16 * k, c = 4 * (threadIdx.x & 15);
#pragma unroll
        for (int j = 0; j < 4; j++) dv[k][j] = sv[k][j] = 0;
        if (r < t.h && c + 4 <= t.w) {
            load4(d + (size_t)(t.y0 + r) * P.dstride + t.x0 + c, dv[k]);
            load4(s + (size_t)(t.y0 + r) * P.sstride + t.x0 + c, sv[k]);
        } else if (r < t.h && c < t.w) {
            for (int j = 0; j < t.w - c; j++)
                dv[k][j] = d[(size_t)(t.y0 + r) * P.dstride + t.x0 + c + j],
                sv[k][j] = s[(size_t)(t.y0 + r) * P.sstride + t.x0 + c + j];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int e = dv[k][j] - sv[k][j];
            ps += (uint32_t)dv[k][j];
            pe += (uint32_t)(e * e);
        }
    if (P.dxp) // the dx plane the resident self-guided search reads (one 8-B store per chunk; rows padded to 64)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int r = (threadIdx.x >> 4) + 16 * k, c = 4 * (threadIdx.x & 15);
            if (r < t.h && c < t.w)
                *(uint2 *)(P.dxp + (size_t)(t.y0 + r) * P.fstride + t.x0 + c) =
                    make_uint2(pack2(dv[k][0] - sv[k][0], dv[k][1] - sv[k][1]), pack2(dv[k][2] - sv[k][2], dv[k][3] - sv[k][3]));
        }
    const unsigned long long tsum = wave_sum_u32_wide(ps), tsse = wave_sum_u32_wide(pe);
    if ((threadIdx.x & 63) == WAVE_LAST) {
        atomicAdd(&sum[t.unit], tsum);
        atomicAdd(&sse[t.unit], tsse);
    }
    PROF_END(tk);
}

#ifndef SVTGPU_SG_NC
#define SVTGPU_SG_NC 7
#endif
constexpr int SG_NC = SVTGPU_SG_NC; // candidates per self-guided descent pass (7: a depth-3 outcome tree)
static_assert(SG_NC == 3 || SG_NC == 7 || SG_NC == 15, "a complete outcome tree of at most 32 nodes");

// ---------------------------------------------------------------------------------------------
// Wiener statistics on the matrix cores.  Output per tile (unchanged layout): [pair (c1 <= c2)][r1 * 7 + r2] H
// blocks, then [c * 7 + r] M -- raw sums of svt_av1_compute_stats (EbRestorationPick.c:671/708) before the
// bit-depth division.
//
// Per pixel p the feature vector F_p holds the WIN x WIN window Y[r][c] = D[i + o + r][j + o + c] (D = dgd - avg
// with a 3-pixel edge-clamped apron) and X = src - avg; the tile's Gram matrix G = sum_p F_p F_p^T contains every
// H entry and M.  Exact integers on v_mfma_i32_16x16x64_i8: each value v in [-1023, 1023] splits into
// v = 32 * hi + lo with hi = v >> 5 in [-32, 31] and lo = v & 31, so G = 1024 HH + 32 (HL + LH) + LL with three i32
// accumulators per 16 x 16 feature block (|partials| <= 4096 px * 1024 < 2^31).  K = the 64 pixels of one tile row
// per MFMA; the 4 waves take rows i = w (mod 4); only the upper feature blocks (mb <= nb) are computed.
// Operands come straight from two byte planes (hi, lo) of D in LDS: lane l of feature block fb holds feature
// 16 fb + (l & 15) for pixels 16 (l >> 4) .. +15 of the row (the probed gfx950 layout A[m = l & 15][k = 16 (l >> 4)
// + j], B[k][n = l & 15], D[4 (l >> 4) + r][l & 15]); the window's column offset is an unaligned byte start, read
// as 5 dwords and realigned with v_alignbyte.  Per wave the three accumulators fold into one i32 (|G_wave| <=
// 1024 px * 1023^2 < 2^31), the four wave partials meet in LDS in i64 and scatter into the output layout.
// ---------------------------------------------------------------------------------------------
typedef int v4i32 __attribute__((ext_vector_type(4)));
// LDS row stride of the byte planes (70 used + realign slack): 19 dwords, so the rows a feature block's lanes read
// (<= 4 rows at dword offsets 4 g + {0, 1}) fall in distinct banks of each 32-lane group -- with 18 the rows two
// apart met in one bank (1.75-2 LDS cycles per read instead of 1.0-1.25)
constexpr int SM_RS = 76;
constexpr int SM_DROWS = 70, SM_XROWS = 64; // D rows (tile + 2 x 3 apron), X rows
constexpr int SM_PLANE = (SM_DROWS + SM_XROWS) * SM_RS + 16; // one byte plane: D rows, then X rows, + read slack

template <int WIN>
struct StatsCfg {
    static constexpr int HALF = WIN / 2, NPAIR = WIN * (WIN + 1) / 2, NF = WIN * WIN + 1;
    static constexpr int NFB = (NF + 15) / 16, NB = NFB * (NFB + 1) / 2, NVAL = (NPAIR + 1) * 49;
};

template <typename T, int WIN>
__global__ __launch_bounds__(256) void wiener_stats_kernel(const SearchArgs A, int tile_begin,
                                                           const unsigned long long *sum, long long *part,
                                                           unsigned long long *tk) {
    PROF_BEGIN(tk);
    using C = StatsCfg<WIN>;
    constexpr int NFB = C::NFB, NB = C::NB, NVAL = C::NVAL;
    // byte planes (hi, lo) during the products; afterwards the wave partials [4][NB][4][64] i32 and the output
    constexpr int LDS_STAGE = 2 * SM_PLANE, LDS_RED = 4 * NB * 256 * 4 + NVAL * 8;
    __shared__ __align__(16) uint8_t lds[LDS_STAGE > LDS_RED ? LDS_STAGE : LDS_RED];
    const int        tl = xcd_swizzle(blockIdx.x, gridDim.x);
    const Tile       t = A.tiles[tile_begin + tl];
    const PlaneArgs &P = A.pl[t.plane];
    const URect      u = A.units[t.unit];
    const long long  area = (long long)(u.h_end - u.h_start) * (u.v_end - u.v_start);
    const int        avg  = (int)(sum[t.unit] / (unsigned long long)area);
    const T         *d = (const T *)P.dgd, *s = (const T *)P.src;
    const int        tid = threadIdx.x, o = 3 - C::HALF;
    // ---- stage: D rows 0 .. h+5 (columns 0 .. w+5, edge-clamped), then X rows 0 .. h-1, as hi / lo bytes ----
    {
        uint32_t *hi = (uint32_t *)lds, *lo = (uint32_t *)(lds + SM_PLANE);
        // (the frame search's tiles are 4-aligned; the per-unit shim's last tile may end inside a group of 4 -- its
        // source reads stay inside the staged window and the products mask those pixels, below)
        const int ng = (t.w + 6 + 3) >> 2, nd = (t.h + 6) * ng, gw = (t.w + 3) >> 2, nx = t.h * gw;
        for (int it = tid; it < nd + nx; it += 256) {
            int v[4], row;
            if (it < nd) {
                row          = it / ng;
                const int g4 = it - row * ng, y = t.y0 + row - 3, x = t.x0 + 4 * g4 - 3;
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = px(d, P.dstride, P.W, P.H, y, x + k) - avg;
                row = row * (SM_RS / 4) + g4;
            } else {
                const int q = it - nd, r = q / gw, g4 = q - r * gw;
                int       sv[4];
                load4(s + (size_t)(t.y0 + r) * P.sstride + t.x0 + 4 * g4, sv);
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = sv[k] - avg;
                row = (SM_DROWS + r) * (SM_RS / 4) + g4;
            }
            uint32_t h4 = 0, l4 = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) h4 |= (uint32_t)(v[k] >> 5 & 0xFF) << (8 * k), l4 |= (uint32_t)(v[k] & 31) << (8 * k);
            hi[row] = h4, lo[row] = l4;
        }
    }
    __syncthreads();
    // ---- products ----
    const int w = tid >> 6, l = tid & 63, g = l >> 4;
    int       fdw[NFB], fsh[NFB]; // dword address (row 0) and byte shift of this lane's feature per block
    uint32_t  fmask[NFB];         // 0: padding feature
#pragma unroll
    for (int fb = 0; fb < NFB; fb++) {
        const int f = 16 * fb + (l & 15);
        int       byte = 0;
        fmask[fb]      = 0xFFFFFFFFu;
        if (f < WIN * WIN) {
            const int r = f / WIN, c = f - r * WIN;
            byte        = (o + r) * SM_RS + 16 * g + c + o;
        } else if (f == WIN * WIN) {
            byte = SM_DROWS * SM_RS + 16 * g;
        } else {
            fmask[fb] = 0;
        }
        fdw[fb] = byte >> 2, fsh[fb] = byte & 3;
    }
    uint32_t cmask[4]; // pixel columns 16 g + 4 q .. +3 inside the tile
#pragma unroll
    for (int q = 0; q < 4; q++) { // byte j = pixel column 16 g + 4 q + j
        const int c = 16 * g + 4 * q;
        cmask[q]    = c + 4 <= t.w ? 0xFFFFFFFFu : c >= t.w ? 0u : 0xFFFFFFFFu >> (8 * (4 - (t.w - c)));
    }
    v4i32 hh[NB], ll[NB], hl[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) hh[b] = ll[b] = hl[b] = v4i32{0, 0, 0, 0};
    const uint32_t *H32 = (const uint32_t *)lds, *L32 = (const uint32_t *)(lds + SM_PLANE);
    for (int i = w; i < t.h; i += 4) {
        v4i32 fh[NFB], fl[NFB];
#pragma unroll
        for (int fb = 0; fb < NFB; fb++) {
            const int rowdw = fdw[fb] + i * (SM_RS / 4), shb = fsh[fb] * 8;
            uint32_t  a[5], b5[5];
#pragma unroll
            for (int k = 0; k < 5; k++) a[k] = H32[rowdw + k], b5[k] = L32[rowdw + k];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t m = cmask[q] & fmask[fb];
                fh[fb][q] = (int)(__builtin_amdgcn_alignbyte(a[q + 1], a[q], shb >> 3) & m);
                fl[fb][q] = (int)(__builtin_amdgcn_alignbyte(b5[q + 1], b5[q], shb >> 3) & m);
            }
        }
        int b = 0;
#pragma unroll
        for (int mb = 0; mb < NFB; mb++)
#pragma unroll
            for (int nb = mb; nb < NFB; nb++, b++) {
                hh[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fh[mb], fh[nb], hh[b], 0, 0, 0);
                ll[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fl[mb], fl[nb], ll[b], 0, 0, 0);
                hl[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fh[mb], fl[nb], hl[b], 0, 0, 0);
                hl[b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fl[mb], fh[nb], hl[b], 0, 0, 0);
            }
    }
    __syncthreads(); // the byte planes are no longer read
    // ---- wave partials -> LDS [w][b][r][lane] ----
    int *red = (int *)lds;
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) red[((w * NB + b) * 4 + r) * 64 + l] = 1024 * hh[b][r] + 32 * hl[b][r] + ll[b][r];
    long long *out = (long long *)(lds + 4 * NB * 256 * 4);
    for (int k = tid; k < NVAL; k += 256) out[k] = 0;
    __syncthreads();
    // ---- totals and scatter into the output layout (each unordered feature pair once) ----
    constexpr int NW = WIN * WIN;
    for (int e = tid; e < NB * 256; e += 256) {
        const int b = e >> 8, r = (e >> 6) & 3, ln = e & 63;
        int       mb = 0, bb = b;
        while (bb >= NFB - mb) bb -= NFB - mb, mb++;
        const int nb = mb + bb;
        const int fm = 16 * mb + 4 * (ln >> 4) + r, fn = 16 * nb + (ln & 15);
        if (mb == nb && fm > fn) continue;
        const long long v = (long long)red[((0 * NB + b) * 4 + r) * 64 + ln] + red[((1 * NB + b) * 4 + r) * 64 + ln] +
                            red[((2 * NB + b) * 4 + r) * 64 + ln] + red[((3 * NB + b) * 4 + r) * 64 + ln];
        if (fm < NW && fn < NW) {
            int r1 = fm / WIN, c1 = fm - r1 * WIN, r2 = fn / WIN, c2 = fn - r2 * WIN;
            if (c1 > c2) {
                const int tr = r1, tc = c1;
                r1 = r2, c1 = c2, r2 = tr, c2 = tc;
            }
            const int pair = c1 * WIN - c1 * (c1 - 1) / 2 + (c2 - c1);
            out[pair * 49 + r1 * 7 + r2] = v;
            if (c1 == c2) out[pair * 49 + r2 * 7 + r1] = v;
        } else if (fm < NW && fn == NW) {
            const int r1 = fm / WIN, c1 = fm - r1 * WIN;
            out[C::NPAIR * 49 + c1 * 7 + r1] = v;
        }
    }
    __syncthreads();
    long long *dst = part + (size_t)tl * NVAL;
    for (int k = tid; k < NVAL; k += 256) dst[k] = out[k];
    PROF_END(tk);
}

// per unit: sum the tile partials (tiles of a unit are contiguous in the tile list)
__global__ void reduce_parts_kernel(const long long *part, const int32_t *unit_tile0, int tile_begin, int nvals,
                                    long long *out, unsigned long long *tk) {
    PROF_BEGIN(tk);
    const int u = blockIdx.x, t0 = unit_tile0[u] - tile_begin, t1 = unit_tile0[u + 1] - tile_begin;
    for (int k = blockIdx.y * blockDim.x + threadIdx.x; k < nvals; k += gridDim.y * blockDim.x) {
        long long s = 0;
        for (int t = t0; t < t1; t++) s += part[(size_t)t * nvals + k];
        out[(size_t)u * nvals + k] = s;
    }
    PROF_END(tk);
}

// ---------------------------------------------------------------------------------------------
// Wiener trial: SSE of every tile of a unit with a pending candidate, filtered with the unit's candidate taps
// (hfilter[8], vfilter[8]).  The advance kernel lists those tiles (items); a fixed grid of persistent workgroups
// takes contiguous runs of the list (XCD-aware, so neighbouring tiles share an L2) and software-pipelines them:
// the next tile's global loads (its tile record, mode, cached pass or CDEF pixels, source pixels) are issued into
// registers right after the current tile is staged in LDS, and land while the current tile is filtered.  Both
// passes run on packed int16 pairs with v_dot2_i32_i16, two outputs per lane: the staged tile (columns
// x0-4 .. x0+w+3, rows y0-3 .. y0+h+3) is read as aligned column pairs, the horizontal output is stored as row
// pairs.  Fixed lane mappings (no runtime divisions): staging in 18 groups of 4 pixels per row, the horizontal
// pass as 32 column pairs x 8 rows per step, the vertical pass as 64 columns x 4 row pairs per step.
// ---------------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------------
// self-guided filters of every searched ep of a tile.  The 3x3 and 5x5 box sums do not depend on ep and stay in
// registers; per ep the A/B maps (packed B << 9 | A) go to LDS and the filters to HBM as g = flt - (dgd << 4), the
// projection's operand (int16: |g| < 2^15), so the resident search (sgr_res_kernel) needs no dgd to form it.
// ---------------------------------------------------------------------------------------------
constexpr int SG_V = 70, SG_B = 66, SG_NT = 1024, SG_NQ = (SG_B * SG_B + SG_NT - 1) / SG_NT;
constexpr int SG_NQ2 = ((SG_B + 1) / 2 * SG_B + SG_NT - 1) / SG_NT; // r = 2 map positions per lane (odd rows only)

// A, B of a self-guided pass from its box sums with 24-bit multiplies where the operands provably fit:
// b <= 25*1023 >> (bd-8) < 2^24; a*n <= 1.64e6*25 < 2^32 with a < 2^24; (256-A)*sum <= 255*25575 < 2^24 and
// times one_by_x (<= 455) < 2^32.  Only p*s wraps like the reference's u32 product and keeps the full multiply.
// Split in two so that a lane's table lookups (A = x_by_xplus1[z]) of all its positions are issued together:
// sgr_z gives the clamped table index, sgr_ab_pack the packed map word (B << 9 | A).  sh = bd - 8.
__device__ inline uint32_t sgr_z(int sum, int sq, int n, int s, int sh) {
    const uint32_t a = (uint32_t)((sq + ((1 << (2 * sh)) >> 1)) >> (2 * sh));
    const uint32_t b = (uint32_t)((sum + ((1 << sh) >> 1)) >> sh);
    const uint32_t an = __umul24(a, (uint32_t)n), bb = __umul24(b, b);
    const uint32_t p  = an < bb ? 0u : an - bb;
    return min((p * (uint32_t)s + (1u << 19)) >> 20, 255u);
}
__device__ inline int sgr_ab_pack(int A, int sum, int n) {
    const int B = (int)((__umul24(__umul24((uint32_t)(256 - A), (uint32_t)sum), (uint32_t)c_one_by_x[n - 1]) + (1u << 11)) >> 12);
    return (B << 9) | A;
}

template <typename T>
__global__ __launch_bounds__(SG_NT) void sgr_flt_kernel(const SearchArgs A, unsigned long long *tk) {
    PROF_BEGIN(tk);
    // packed B << 9 | A (A <= 256, B < 2^19) of the r = 1 and r = 2 passes, double-buffered over eps: the maps of
    // ep e + 1 are built while ep e is filtered, one barrier per ep
    __shared__ int ab1[2][SG_B * SG_B], ab2[2][SG_B * SG_B];
    __shared__ int      xby[256];
    // the tile with its 3-pixel border lives in ab1[1] until the box sums are taken (ab1[1] is first written by
    // build_ab(1), after the barrier that follows build_ab(0)): 70 KB of LDS, two workgroups per CU
    static_assert(SG_V * SG_V * 2 <= SG_B * SG_B * 4, "tile image fits the aliased map buffer");
    uint16_t *const v = (uint16_t *)ab1[1];
    const Tile       t = A.tiles[xcd_swizzle(blockIdx.x, gridDim.x)];
    const PlaneArgs &P = A.pl[t.plane];
    const T         *d = (const T *)P.dgd;
    for (int i = threadIdx.x; i < (t.h + 6) * (t.w + 6); i += SG_NT) {
        const int r = i / (t.w + 6), c = i % (t.w + 6);
        v[r * SG_V + c] = (uint16_t)px(d, P.dstride, P.W, P.H, t.y0 + r - 3, t.x0 + c - 3);
    }
    if (threadIdx.x < 256) xby[threadIdx.x] = c_x_by_xplus1[threadIdx.x];
    __syncthreads();
    const uint16_t *v0 = v + 3 * SG_V + 3;
    // The box sums read a row's 3 / 5 samples as aligned dword pairs and a funnel shift (sr_lds_pair) plus one 16-bit
    // read: adjacent 16-bit reads merged by the compiler into one dword / quad read would be misaligned for half the
    // lanes, which the LDS serves far below its rate.  Index a of v (4-B aligned: the int array ab1[1]).
    auto lds_pair = [&](int a) {
        const uint32_t *w = (const uint32_t *)v + (a >> 1);
        return __builtin_amdgcn_alignbit(w[1], w[0], (a & 1) * 16);
    };
    const int       bw = t.w + 2, nq = (t.h + 2) * bw, nq2 = (t.h + 3) / 2 * bw;
    // the r = 1 map at every position q (map row q / bw = pixel row - 1 .. t.h); the r = 2 map only on the odd pixel
    // rows (-1, 1, ..): dense position i -> map row 2 (i / bw), so no lane idles on the even rows
    int s1[SG_NQ], q1[SG_NQ], s2[SG_NQ2], q2[SG_NQ2], m2q[SG_NQ2];
#pragma unroll
    for (int k = 0; k < SG_NQ; k++) {
        const int q = threadIdx.x + k * SG_NT;
        s1[k] = q1[k] = 0;
        if (q < nq) {
            const int y = q / bw - 1, x = q % bw - 1;
#pragma unroll
            for (int dy = -1; dy <= 1; dy++) {
                const int      a  = (y + dy + 3) * SG_V + x + 3; // sample (y + dy, x) of the tile image
                const uint32_t pr = lds_pair(a - 1);
                const int      p[3] = {(int)(pr & 0xFFFF), (int)(pr >> 16), (int)v[a + 1]};
#pragma unroll
                for (int j = 0; j < 3; j++) s1[k] += p[j], q1[k] += p[j] * p[j];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < SG_NQ2; k++) {
        const int i = threadIdx.x + k * SG_NT, row = i / bw, x = i - row * bw - 1, y = 2 * row - 1;
        s2[k] = q2[k] = 0;
        m2q[k] = i < nq2 ? (y + 1) * bw + x + 1 : -1; // the map index the filters read
        if (i < nq2) {
#pragma unroll
            for (int dy = -2; dy <= 2; dy++) {
                const int      a  = (y + dy + 3) * SG_V + x + 3;
                const uint32_t pa = lds_pair(a - 2), pb = lds_pair(a);
                const int      p[5] = {(int)(pa & 0xFFFF), (int)(pa >> 16), (int)(pb & 0xFFFF), (int)(pb >> 16), (int)v[a + 2]};
#pragma unroll
                for (int j = 0; j < 5; j++) s2[k] += p[j], q2[k] += p[j] * p[j];
            }
        }
    }
    // this lane's pixels: a column of 4 rows (fy0 .. fy0 + 3, fy0 even) at column fx, so the 3-wide map rows a filter
    // reads are loaded and summed once for the column (6 rows for the r = 1 filter, 3 for r = 2) instead of once
    // per pixel.  The division by the tile width is done once here, not per ep
    const int fr = (int)threadIdx.x / t.w, fx = (int)threadIdx.x - fr * t.w, fy0 = 4 * fr;
    const bool fon = fy0 < t.h;
    int        pix[4];
#pragma unroll
    for (int k = 0; k < 4; k++) pix[k] = fon && fy0 + k < t.h ? v0[(fy0 + k) * SG_V + fx] : 0;
    const int   fq  = fx + 1;                                             // map column of the lane's pixels
    const size_t fo = (size_t)(t.y0 + fy0) * P.fstride + t.x0 + fx;       // filter-plane offset of row fy0
    const size_t pn = (size_t)P.fstride * P.H;
    const int sh = P.bd - 8;
    auto build_ab = [&](int e) { // A/B maps of ep index e into buffer e & 1
        const int ep = P.eps[e], r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
        int      *m1 = ab1[e & 1], *m2 = ab2[e & 1];
        if (r1 && P.f1e[e] == e) { // r = 1 (3x3) at every map position
            const int sp = c_sgr_s[ep][1];
            uint32_t  z[SG_NQ];
            int       a[SG_NQ];
#pragma unroll
            for (int k = 0; k < SG_NQ; k++) z[k] = sgr_z(s1[k], q1[k], 9, sp, sh);
#pragma unroll
            for (int k = 0; k < SG_NQ; k++) a[k] = xby[z[k]]; // the lookups in flight together
#pragma unroll
            for (int k = 0; k < SG_NQ; k++) {
                const int q = threadIdx.x + k * SG_NT;
                if (q < nq) m1[q] = sgr_ab_pack(a[k], s1[k], 9);
            }
        }
        if (r0) { // r = 2 (5x5) on the odd rows
            const int sp = c_sgr_s[ep][0];
            uint32_t  z[SG_NQ2];
            int       a[SG_NQ2];
#pragma unroll
            for (int k = 0; k < SG_NQ2; k++) z[k] = sgr_z(s2[k], q2[k], 25, sp, sh);
#pragma unroll
            for (int k = 0; k < SG_NQ2; k++) a[k] = xby[z[k]];
#pragma unroll
            for (int k = 0; k < SG_NQ2; k++)
                if (m2q[k] >= 0) m2[m2q[k]] = sgr_ab_pack(a[k], s2[k], 25);
        }
    };
    build_ab(0);
    __syncthreads();
    for (int e = 0; e < P.ne; e++) {
        if (e + 1 < P.ne) build_ab(e + 1);
        const int  ep = P.eps[e], r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
        const int *ab1e = ab1[e & 1], *ab2e = ab2[e & 1];
        int16_t  *f0g = P.flt + (size_t)e * 2 * pn, *f1g = f0g + pn;
        if (fon) {
            // 3-wide sums of map row ry (pixel-row coordinates -1 .. t.h; rows past the tile are clamped, their
            // pixels are not stored): packed (B << 9 | A) and A-only sums of the row triple and of its centre
            struct Row { int s, sa, c, ca; };
            auto row = [&](const int *M, int ry) {
                const int *Q = M + (min(ry, t.h) + 1) * bw + fq;
                const int  l = Q[-1], c = Q[0], r = Q[1];
                Row        w;
                w.c = c, w.ca = c & 511, w.s = l + c + r, w.sa = (l & 511) + w.ca + (r & 511);
                return w;
            };
            const int nk = min(4, t.h - fy0);
            if (r0) { // r = 2 maps exist on odd rows: fy0 - 1, fy0 + 1, fy0 + 3
                Row up = row(ab2e, fy0 - 1);
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int k = 2 * h;
                    if (k >= nk) break;
                    const Row dn = row(ab2e, fy0 + k + 1);
                    { // even row fy0 + k: rows above and below, weights 6 (centres) and 5 (corners)
                        const int c6 = up.c + dn.c, a6 = up.ca + dn.ca;
                        const int c5 = up.s - up.c + dn.s - dn.c, a5 = up.sa - up.ca + dn.sa - dn.ca;
                        const int aa = a6 * 6 + a5 * 5, bb = ((c6 - a6) >> 9) * 6 + ((c5 - a5) >> 9) * 5;
                        f0g[fo + (size_t)k * P.fstride] =
                            (int16_t)((((int)__umul24((uint32_t)aa, (uint32_t)pix[k]) + bb + (1 << 8)) >> 9) - (pix[k] << 4));
                    }
                    if (k + 1 < nk) { // odd row fy0 + k + 1: its own row, weights 6 (centre) and 5 (sides)
                        const int a6 = dn.ca, a5 = dn.sa - dn.ca;
                        const int aa = a6 * 6 + a5 * 5, bb = ((dn.c - a6) >> 9) * 6 + ((dn.s - dn.c - a5) >> 9) * 5;
                        f0g[fo + (size_t)(k + 1) * P.fstride] =
                            (int16_t)((((int)__umul24((uint32_t)aa, (uint32_t)pix[k + 1]) + bb + (1 << 7)) >> 8) -
                                      (pix[k + 1] << 4));
                    }
                    up = dn;
                }
            }
            if (r1 && P.f1e[e] == e) { // an ep sharing an earlier slot's r = 1 filter reads that plane
                Row pv = row(ab1e, fy0 - 1), cu = row(ab1e, fy0);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (k >= nk) break;
                    const Row nx = row(ab1e, fy0 + k + 1);
                    // weights 4: the row triple and the centres above/below; 3: the four corners
                    const int c4 = cu.s + pv.c + nx.c, a4 = cu.sa + pv.ca + nx.ca;
                    const int c3 = pv.s - pv.c + nx.s - nx.c, a3 = pv.sa - pv.ca + nx.sa - nx.ca;
                    const int aa = a4 * 4 + a3 * 3, bb = ((c4 - a4) >> 9) * 4 + ((c3 - a3) >> 9) * 3;
                    f1g[fo + (size_t)k * P.fstride] =
                        (int16_t)((((int)__umul24((uint32_t)aa, (uint32_t)pix[k]) + bb + (1 << 8)) >> 9) - (pix[k] << 4));
                    pv = cu, cu = nx;
                }
            }
        }
        __syncthreads(); // ep e + 2 rewrites this ep's buffer; ep e + 1's maps are complete
    }
    PROF_END(tk);
}

typedef short v2i16s __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pk_sub16(uint32_t a, uint32_t b) { // per-half a - b mod 2^16
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2i16s, a) - __builtin_bit_cast(v2i16s, b));
}

// SSE of the chosen self-guided output (apply_selfguided_restoration: projection, int16 wrap, clip)
template <typename T>
__global__ __launch_bounds__(256) void sgr_sse_kernel(const SearchArgs A, const int32_t *best, unsigned long long *err,
                                                      unsigned long long *tk) {
    PROF_BEGIN(tk);
    const Tile       t = A.tiles[xcd_swizzle(blockIdx.x, gridDim.x)];
    const PlaneArgs &P = A.pl[t.plane];
    const int       *b = best + t.unit * 4; // {ep index, ep, xq0, xq1}
    const int        e = b[0], ep = b[1], xq0 = b[2], xq1 = b[3], r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
    const T         *d = (const T *)P.dgd, *s = (const T *)P.src;
    const size_t     pn = (size_t)P.fstride * P.H;
    const int16_t   *f0 = P.flt + (size_t)e * 2 * pn, *f1 = P.flt + (size_t)(e >= 0 ? P.f1e[e] : e) * 2 * pn + pn;
    const int        maxv = (1 << P.bd) - 1;
    unsigned long long acc = 0;
    // 4-sample chunks as in unit_sums_kernel: chunk k of this lane is row (threadIdx.x >> 4) + 16 k, columns
    // 4 (threadIdx.x & 15) .. + 3
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int r = (threadIdx.x >> 4) + 16 * k, c = 4 * (threadIdx.x & 15);
        if (r >= t.h || c >= t.w) continue;
        const int    y = t.y0 + r, x = t.x0 + c;
        const size_t o = (size_t)y * P.fstride + x;
        int          dv[4], sv[4], g0[4] = {0, 0, 0, 0}, g1[4] = {0, 0, 0, 0};
        const int    nv = min(4, t.w - c); // a partial chunk at a crop width that is not a multiple of 4
        if (nv == 4) {
            load4(d + (size_t)y * P.dstride + x, dv);
            load4(s + (size_t)y * P.sstride + x, sv);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++)
                dv[j] = j < nv ? (int)d[(size_t)y * P.dstride + x + j] : 0,
                sv[j] = j < nv ? (int)s[(size_t)y * P.sstride + x + j] : 0;
        }
        if (r0 > 0) load4s(f0 + o, g0); // g = flt - u planes; rows padded to 64 samples
        if (r1 > 0) load4s(f1 + o, g1);
        uint32_t e2 = 0; // 4 squared errors of at most 1023^2
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (j >= nv) break;
            const int u = dv[j] << 4;
            int       v = u << 7;
            if (r0 > 0) v += xq0 * g0[j];
            if (r1 > 0) v += xq1 * g1[j];
            const int16_t w  = (int16_t)((v + (1 << 10)) >> 11);
            const int     ov = min(max((int)w, 0), maxv);
            e2 += (uint32_t)((ov - sv[j]) * (ov - sv[j]));
        }
        acc += e2;
    }
    const unsigned long long at = wave_sum(acc);
    if ((threadIdx.x & 63) == WAVE_LAST) atomicAdd(&err[t.unit], at);
    PROF_END(tk);
}

// =============================================================================================
// the reference's sequential logic (host), and the coordinate descent (host and device)
// =============================================================================================
constexpr int64_t TAP_SCALE = (int64_t)1 << 16;
constexpr int     FILT_STEP = 128;

__host__ __device__ inline int wrap_index(int i, int win) { return i >= (win >> 1) + 1 ? win - 1 - i : i; }
__host__ __device__ inline int64_t abs64(int64_t v) { return v < 0 ? -v : v; }

__device__ int linsolve_wiener(int n, int64_t *A, int stride, int64_t *b, int32_t *x) { // EbRestorationPick.c:766-803
    for (int k = 0; k < n - 1; k++) {
        for (int i = n - 1; i > k; i--)
            if (abs64(A[(i - 1) * stride + k]) < abs64(A[i * stride + k])) {
                for (int j = 0; j < n; j++) {
                    const int64_t t = A[i * stride + j];
                    A[i * stride + j] = A[(i - 1) * stride + j], A[(i - 1) * stride + j] = t;
                }
                const int64_t t = b[i];
                b[i] = b[i - 1], b[i - 1] = t;
            }
        for (int i = k; i < n - 1; i++) {
            if (A[k * stride + k] == 0) return 0;
            const int64_t c = A[(i + 1) * stride + k], cd = A[k * stride + k];
            for (int j = 0; j < n; j++) A[(i + 1) * stride + j] -= c / 256 * A[k * stride + j] / cd * 256;
            b[i + 1] -= c * b[k] / cd;
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        if (A[i * stride + i] == 0) return 0;
        int64_t c = 0;
        for (int j = i + 1; j <= n - 1; j++) c += A[i * stride + j] * x[j] / TAP_SCALE;
        x[i] = (int32_t)(TAP_SCALE * (b[i] - c) / A[i * stride + i]);
    }
    return 1;
}

// Shared-memory workspace of the per-unit Wiener decomposition (one workgroup per unit)
struct WienerSolveLds {
    int64_t M[49], H[49 * 49];
    int64_t accA[4], accB[16], accP, accQ;
    int32_t a[7], b[7], ab[49];
};

// update_a_sep_sym (solve_b = false) / update_b_sep_sym (EbRestorationPick.c:805-904), H viewed as hc[r][c].
// Every term of the reference's A / B sums is formed exactly as the reference forms it; the integer sums are
// split over the lanes (5 lanes per B cell) and combined with LDS atomics, which is exact.
__device__ void update_sep_sym(bool solve_b, int win, WienerSolveLds &L) {
    const int win2 = win * win, h1 = (win >> 1) + 1, tid = threadIdx.x;
    if (tid < 16) L.accB[tid] = 0;
    if (tid < 4) L.accA[tid] = 0;
    __syncthreads();
    auto hc = [&](int r, int c) { return L.H[(r / win) * win * win2 + (r % win) * win + c]; };
    if (tid < win2) {
        const int     i = tid / win, j = tid % win;
        const int64_t t = solve_b ? L.M[i * win + j] * L.a[j] / TAP_SCALE : L.M[i * win + j] * L.b[i] / TAP_SCALE;
        atomicAdd((unsigned long long *)&L.accA[solve_b ? wrap_index(i, win) : wrap_index(j, win)], (unsigned long long)t);
    }
    constexpr int SL = 5;
    const int     cell = tid / SL;
    if (cell < win2) {
        const int c0 = cell / win, c1 = cell % win;
        int64_t   sum = 0;
        for (int q = tid % SL; q < win2; q += SL) {
            const int o0 = q / win, o1 = q % win;
            if (!solve_b) // cell (k, l), terms over (i, j)
                sum += hc(o1 * win + o0, c0 * win2 + c1) * L.b[o0] / TAP_SCALE * L.b[o1] / TAP_SCALE;
            else // cell (i, j), terms over (k, l)
                sum += hc(c0 * win + c1, o0 * win2 + o1) * L.a[o0] / TAP_SCALE * L.a[o1] / TAP_SCALE;
        }
        const int idx = wrap_index(c1, win) * h1 + wrap_index(c0, win); // (l, k) resp. (j, i)
        atomicAdd((unsigned long long *)&L.accB[idx], (unsigned long long)sum);
    }
    __syncthreads();
    if (tid == 0) {
        int64_t *A = L.accA, *B = L.accB;
        int32_t  S[7];
        const int64_t last = A[h1 - 1];
        for (int i = 0; i < h1 - 1; i++) A[i] -= last * 2 + B[i * h1 + h1 - 1] - 2 * B[(h1 - 1) * h1 + (h1 - 1)];
        for (int i = 0; i < h1 - 1; i++)
            for (int j = 0; j < h1 - 1; j++)
                B[i * h1 + j] -= 2 * (B[i * h1 + (h1 - 1)] + B[(h1 - 1) * h1 + j] - 2 * B[(h1 - 1) * h1 + (h1 - 1)]);
        if (linsolve_wiener(h1 - 1, B, h1, A, S)) {
            S[h1 - 1] = (int32_t)TAP_SCALE;
            for (int i = h1; i < win; i++) {
                S[i] = S[win - 1 - i];
                S[h1 - 1] -= 2 * S[i];
            }
            int32_t *dst = solve_b ? L.b : L.a;
            for (int i = 0; i < win; i++) dst[i] = S[i];
        }
    }
    __syncthreads();
}

__constant__ int c_tap_min[3] = {-5, -23, -17}, c_tap_max[3] = {10, 8, 46};

__device__ void finalize_sym_filter(int win, const int32_t *f, int16_t *fi) { // EbRestorationPick.c:977-1006
    for (int i = 0; i < (win >> 1); i++) {
        const int64_t n = (int64_t)f[i] * FILT_STEP;
        fi[i]           = (int16_t)(n < 0 ? (n - TAP_SCALE / 2) / TAP_SCALE : (n + TAP_SCALE / 2) / TAP_SCALE);
    }
    auto clip = [](int v, int t) { return (int16_t)min(max(v, c_tap_min[t]), c_tap_max[t]); };
    if (win == 7) {
        fi[0] = clip(fi[0], 0), fi[1] = clip(fi[1], 1), fi[2] = clip(fi[2], 2);
    } else {
        fi[2] = clip(fi[1], 2), fi[1] = clip(fi[0], 1), fi[0] = 0;
    }
    fi[6] = fi[0], fi[5] = fi[1], fi[4] = fi[2];
    fi[3] = (int16_t)(-2 * (fi[0] + fi[1] + fi[2]));
    fi[7] = 0;
}

// compute_score (EbRestorationPick.c:1008-1040): the P and Q sums split over the lanes
__device__ int64_t compute_score(int win, WienerSolveLds &L, const int16_t *vf, const int16_t *hf) {
    const int off = (7 - win) >> 1, win2 = win * win, tid = threadIdx.x;
    if (tid == 0) {
        int16_t a[7], b[7];
        a[3] = b[3] = FILT_STEP;
        for (int i = 0; i < 3; i++) {
            a[i] = a[6 - i] = vf[i];
            b[i] = b[6 - i] = hf[i];
            a[3] -= 2 * a[i];
            b[3] -= 2 * b[i];
        }
        for (int k = 0; k < win; k++)
            for (int l = 0; l < win; l++) L.ab[k * win + l] = a[l + off] * b[k + off];
        L.accP = 0, L.accQ = 0;
    }
    __syncthreads();
    if (tid < win2) atomicAdd((unsigned long long *)&L.accP, (unsigned long long)(L.ab[tid] * L.M[tid] / FILT_STEP / FILT_STEP));
    int64_t q = 0;
    for (int t = tid; t < win2 * win2; t += blockDim.x) {
        const int k = t / win2, l = t % win2;
        q += L.ab[k] * L.H[k * win2 + l] * L.ab[l] / FILT_STEP / FILT_STEP / FILT_STEP / FILT_STEP;
    }
    atomicAdd((unsigned long long *)&L.accQ, (unsigned long long)q);
    __syncthreads();
    return (L.accQ - 2 * L.accP) - (L.H[(win2 >> 1) * win2 + (win2 >> 1)] - 2 * L.M[win2 >> 1]);
}

// rates (EbEntropyCoding.c:2876-3022, EbRestorationPick.c:655-668, 1008-1040); host and device (the RD finish runs
// on either)
__host__ __device__ inline int count_quniform(int n, int v) {
    if (n <= 1) return 0;
    const int l = 32 - __builtin_clz((unsigned)(n - 1)), m = (1 << l) - n;
    return v < m ? l - 1 : l;
}
__host__ __device__ inline int count_subexpfin(int n, int k, int v) {
    int count = 0, i = 0, mk = 0;
    for (;;) {
        const int b = i ? k + i - 1 : k, a = 1 << b;
        if (n <= mk + 3 * a) return count + count_quniform(n - mk, v - mk);
        count++;
        if (v >= mk + a) {
            i++;
            mk += a;
        } else
            return count + b;
    }
}
__host__ __device__ inline int refsubexpfin(int n, int k, int ref, int v) {
    n &= 0xFFFF, ref &= 0xFFFF, v &= 0xFFFF;
    const int r = (ref << 1) <= n ? ref : n - 1 - ref, x = (ref << 1) <= n ? v : n - 1 - v; // recentering
    const int rv = x > (r << 1) ? x : x >= r ? (x - r) << 1 : ((r - x) << 1) - 1;
    return count_subexpfin(n, k, rv & 0xFFFF);
}
// WIENER_FILT_TAP{0,1,2}_{MINV,MAXV} (EbDefinitions.h) and the self-guided sets with an r = 0 / r = 1 pass
__host__ __device__ inline int tap_min(int t) { return t == 0 ? -5 : t == 1 ? -23 : -17; }
__host__ __device__ inline int tap_max(int t) { return t == 0 ? 10 : t == 1 ? 8 : 46; }
__host__ __device__ inline bool sgr_r0(int ep) { return ep < 10 || ep > 13; } // c_sgr_r[ep][0] > 0
__host__ __device__ inline bool sgr_r1(int ep) { return ep < 14; }            // c_sgr_r[ep][1] > 0
// unrolled over constant tap indices: on the device the taps stay in registers (a pointer to either filter array,
// indexed in a loop, put the unit on the stack: every evaluation a chain of scratch round trips)
__host__ __device__ inline int wiener_bits(int win, const SvtGpuRestUnit &w, const SvtGpuRestUnit &ref) {
    int bits = 0;
#pragma unroll
    for (int f = 0; f < 2; f++)
#pragma unroll
        for (int t = 0; t < 3; t++) {
            if (t == 0 && win != 7) continue;
            const int a = f ? w.hfilter[t] : w.vfilter[t], r = f ? ref.hfilter[t] : ref.vfilter[t];
            bits += refsubexpfin(tap_max(t) - tap_min(t) + 1, t + 1, r - tap_min(t), a - tap_min(t));
        }
    return bits;
}
__host__ __device__ inline int sgrproj_bits(const SvtGpuRestUnit &s, const SvtGpuRestUnit &ref) {
    int bits = 4;
    if (sgr_r0(s.ep)) bits += refsubexpfin(PRJ_MAX0 - PRJ_MIN0 + 1, 4, ref.xqd[0] - PRJ_MIN0, s.xqd[0] - PRJ_MIN0);
    if (sgr_r1(s.ep)) bits += refsubexpfin(PRJ_MAX1 - PRJ_MIN1 + 1, 4, ref.xqd[1] - PRJ_MIN1, s.xqd[1] - PRJ_MIN1);
    return bits;
}
// RDCOST_DBL (EbRestoration.h:346-347); the library is built with -ffp-contract=off, so host and device round alike
__host__ __device__ inline double rdcost(int rdmult, int64_t bits, int64_t sse) {
    return ((double)bits * rdmult) / (double)(1 << 9) + (double)sse * (1 << 7);
}
// set_default_wiener / set_default_sgrproj (EbRestorationPick.c rsc_on_tile): the first unit's reference
__host__ __device__ inline SvtGpuRestUnit default_wiener() {
    SvtGpuRestUnit r{};
    const int16_t  mid[7] = {3, -7, 15, -22, 15, -7, 3};
    for (int k = 0; k < 7; k++) r.vfilter[k] = r.hfilter[k] = mid[k];
    return r;
}
__host__ __device__ inline SvtGpuRestUnit default_sgrproj() {
    SvtGpuRestUnit r{};
    r.xqd[0] = (PRJ_MIN0 + PRJ_MAX0) / 2, r.xqd[1] = (PRJ_MIN1 + PRJ_MAX1) / 2;
    return r;
}

// Resumable coordinate descent shared by finer_tile_search_wiener_seg (EbRestorationPick.c:1042-1146) and
// finer_search_pixel_proj_error (:320-413): coordinates (f, p) move by -s then +s; at the first step size a
// successful move is repeated; a successful downward move ends the p loop of its filter.
struct Descent {
    int32_t unit = 0, k = 0, ep = 0;                       // owner: global unit, ep index, ep (self-guided)
    int     start = 0, end = 1, nf = 1, p_lo = 0, p_hi = 0; // p in [p_lo, p_hi]
    bool    cont = true;
    // coordinates and bounds packed as int8 fields (taps and xqd fit), so that the device keeps a descent in
    // registers: value (f, p) at bits 8 * (3 f + p) of vals, bounds of p at bits 8 p of lo4 / hi4
    uint64_t vals = 0;
    uint32_t lo4 = 0, hi4 = 0, skipm = 0;
    __host__ __device__ int  val(int f_, int p_) const { return (int8_t)(vals >> (8 * (3 * f_ + p_))); }
    __host__ __device__ void set_val(int f_, int p_, int v) {
        const int sh = 8 * (3 * f_ + p_);
        vals         = (vals & ~(0xFFull << sh)) | ((uint64_t)(uint8_t)v << sh);
    }
    __host__ __device__ int  lo(int p_) const { return (int8_t)(lo4 >> (8 * p_)); }
    __host__ __device__ int  hi(int p_) const { return (int8_t)(hi4 >> (8 * p_)); }
    __host__ __device__ void set_bounds(int p_, int l, int h) {
        lo4 = (lo4 & ~(0xFFu << (8 * p_))) | ((uint32_t)(uint8_t)l << (8 * p_));
        hi4 = (hi4 & ~(0xFFu << (8 * p_))) | ((uint32_t)(uint8_t)h << (8 * p_));
    }
    __host__ __device__ void taps(int f_, int *v) const { v[0] = val(f_, 0), v[1] = val(f_, 1), v[2] = val(f_, 2); }
    // state
    int     s = 0, f = 0, p = 0, phase = 0;      // phase 0: minus, 1: after minus, 2: plus
    bool    skip = false, init = true, done = false;
    int64_t err = 0;
    int     mf = 0, mp = 0, md = 0;              // pending move
    __host__ __device__ void begin() { s = start, f = 0, p = p_lo, phase = 0, skip = false, init = true, done = false; }
    // proposes the next candidate (val holds it) or sets done; returns true when a candidate is pending
    __host__ __device__ bool next() {
        if (init) return true;
        for (;;) {
            if (s < end) {
                done = true;
                return false;
            }
            if (f >= nf) {
                s >>= 1, f = 0, p = p_lo, phase = 0, skip = false;
                continue;
            }
            if (p > p_hi) {
                f++, p = p_lo, phase = 0, skip = false;
                continue;
            }
            if (skipm >> p & 1) {
                p++;
                continue;
            }
            if (phase == 0) {
                if (val(f, p) - s >= lo(p)) {
                    set_val(f, p, val(f, p) - s), mf = f, mp = p, md = -s;
                    return true;
                }
                phase = 1;
            }
            if (phase == 1) {
                if (skip) {
                    p = p_hi + 1; // `if (skip) break;` leaves the p loop
                    continue;
                }
                phase = 2;
            }
            if (val(f, p) + s <= hi(p)) {
                set_val(f, p, val(f, p) + s), mf = f, mp = p, md = s;
                return true;
            }
            p++, phase = 0, skip = false;
        }
    }
    __host__ __device__ void report(int64_t e2) { report_outcome(!init && e2 > err, e2); }
    // the state change of report() for a known outcome; the candidate sequence depends only on the outcomes, so
    // a speculative tree of candidates can be built before their errors are known
    __host__ __device__ void report_outcome(bool worse, int64_t e2) {
        if (init) {
            err = e2, init = false;
            return;
        }
        if (worse) {
            set_val(mf, mp, val(mf, mp) - md);
            if (md < 0)
                phase = 1;
            else
                p++, phase = 0, skip = false;
        } else {
            err = e2;
            const bool again = s == start && cont;
            if (md < 0) {
                skip = true;
                if (!again) phase = 1;
            } else if (!again)
                p++, phase = 0, skip = false;
        }
    }
};

__host__ __device__ inline void set_wiener_taps(int16_t *t, const int *v) { // symmetric 7-tap from taps 0..2
    t[0] = t[6] = (int16_t)v[0];
    t[1] = t[5] = (int16_t)v[1];
    t[2] = t[4] = (int16_t)v[2];
    t[3] = (int16_t)(-2 * (v[0] + v[1] + v[2]));
    t[7] = 0;
}

// ---------------------------------------------------------------------------------------------
// The Wiener descent of one unit per workgroup with the whole unit resident on the CU (default).
// finer_tile_search_wiener_seg (EbRestorationPick.c:1042-1146) evaluates ~40 candidates one after the other, each
// over every pixel of the unit; the critical path of the search is that chain for the largest unit.  Here nothing
// of a candidate touches global memory:
//   * 1024 lanes; lane = (column pair cp, row segment sg) of the unit: output columns x = 2cp, 2cp+1, rows
//     [sg*R, sg*R+R).  A wave holds 64 consecutive column pairs of one segment, so per-segment control is uniform;
//   * the lane's source pixels stay in registers (one packed (x, x+1) pair per row);
//   * the edge-clamped CDEF window of the unit (rows -3..h+2, columns -4..w+5, 16-bit) is staged into LDS once
//     when it fits; larger units (the frame's bottom unit row, 256 x 376 at 4K) read it from global memory, where
//     only this workgroup touches it (L2-resident);
//   * per candidate every lane walks its rows with a rolling window of four vertical pairs of the horizontal pass
//     per column (the rows y-3 .. y+4 the vertical pass needs), computing one new pair of horizontal rows per pair
//     of output rows: 4 v_dot2 per horizontal and per vertical output, the add-source term folded into the centre
//     taps, the SSE as one v_dot2 of the packed (out - src) pair with itself;
//   * one workgroup barrier per candidate (one-part units): the SSE reduction; every wave then steps its own copy of
//     the descent (Descent::report / next, exactly as the other Wiener paths) in scalar registers and takes the next
//     candidate's taps from it.  Row-part units (and SVTGPU_WR_CLASSIC=1) keep two barriers: lane 0 exchanges the
//     parts' SSEs, steps the descent and writes the taps to LDS.
// The candidate count per unit is bounded (WR_MAX_ROUNDS; a descent always ends far earlier): on overflow the
// descent stops and *status is set, which search_frame reports as SVTGPU_ERR_HIP.
// ---------------------------------------------------------------------------------------------
constexpr int WR_NT = 1024, WR_RMAX = 32, WR_MAX_ROUNDS = 4096;
constexpr int WR_LDS_CAP = 152 * 1024; // largest CDEF window kept in LDS (bytes); larger units read global memory

// geometry of a unit in the lane layout: column-pair slots per segment (a multiple of 64), segments, rows per segment
struct WrGeo {
    int cpw, nseg, R;
};
__host__ __device__ inline WrGeo wr_geo(int w, int h) {
    WrGeo g;
    g.cpw  = (((w + 1) >> 1) + 63) & ~63;
    g.nseg = WR_NT / g.cpw;
    g.R    = (h + g.nseg - 1) / g.nseg;
    return g;
}
__host__ __device__ inline int wr_window_bytes(int w, int h) { return (h + 6) * ((w + 10) >> 1) * 4; }
// LDS mode: the window in LDS and the source rows in registers; else both are read from global memory per candidate
__host__ __device__ inline bool wr_lds_mode(int w, int h, int lds_cap) {
    return wr_window_bytes(w, h) <= lds_cap && wr_geo(w, h).R <= WR_RMAX;
}
// A workgroup's share of a unit: rows [y0, y1) of unit `unit`.  A unit too large for one CU's LDS and registers (the
// frame's bottom unit row: 256 x 376 at 4K) is cut into `nparts` row parts on as many workgroups; each evaluates every
// candidate over its rows, the parts' SSEs meet through words in uncached memory (xch[2 * (first + part) + parity]:
// {round << 48 | partial SSE}, double-buffered by round parity), and every part takes the same descent step.  The
// parts of a unit are adjacent in the launch order and there are far fewer parted workgroups than CUs, so a waiting
// part's partner is always dispatched; the wait is bounded all the same (status bit 2).
struct WrItem {
    int32_t unit, y0, y1, part, nparts, first; // first: the item index of part 0 (exchange slots)
};
constexpr int WR_MAX_PARTS = 4;

// the 5 packed sample pairs of window row r (unit rows -3.., columns x-4 .. x+5) for output columns x, x+1
template <typename T, bool LDSW>
__device__ inline void wr_fetch(const uint32_t *win, int ws, const PlaneArgs &P, int ux, int uy, int hw, int xc, int r,
                                uint32_t *p) {
    r = min(r, hw - 1); // rows past the window only feed outputs that are never used
    if constexpr (LDSW) {
        const uint32_t *q = win + r * ws + (xc >> 1);
#pragma unroll
        for (int k = 0; k < 5; k++) p[k] = q[k];
    } else {
        const T  *d  = (const T *)P.dgd;
        const int fy = min(max(uy - 3 + r, 0), P.H - 1), fx = ux + xc - 4;
        const T  *row = d + (size_t)fy * P.dstride;
        if (fx >= 0 && fx + 10 <= P.W) {
            if constexpr (sizeof(T) == 2) {
                const uint32_t *q = (const uint32_t *)(row + fx);
#pragma unroll
                for (int k = 0; k < 5; k++) p[k] = q[k];
            } else {
                const uint16_t *q = (const uint16_t *)(row + fx);
#pragma unroll
                for (int k = 0; k < 5; k++) p[k] = (uint32_t)(q[k] & 0xFF) | ((uint32_t)(q[k] >> 8) << 16);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const int c0 = min(max(fx + 2 * k, 0), P.W - 1), c1 = min(max(fx + 2 * k + 1, 0), P.W - 1);
                p[k] = (uint32_t)row[c0] | ((uint32_t)row[c1] << 16);
            }
        }
    }
}

// wave-uniform copies (scalar registers) of a 64-bit lane value and of a struct
__device__ __forceinline__ long long readlane64(long long v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l),
                   hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
template <typename S>
__device__ __forceinline__ S uniform(const S &v) {
    static_assert(sizeof(S) % 4 == 0, "whole dwords");
    S r;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(S) / 4); k++)
        ((int *)&r)[k] = __builtin_amdgcn_readfirstlane(((const int *)&v)[k]);
    return r;
}

template <typename T, bool LDSW>
__device__ void wr_run(const SearchArgs &A, const PlaneArgs &P, Descent &D, const uint32_t *win, int ws, int ux,
                       int uy, int w, int h, const WrItem &it, unsigned long long *xch, int *s_mode, int16_t *s_taps,
                       unsigned long long *s_part, int32_t *status, unsigned long long &npx, unsigned long long *stat,
                       bool classic) {
    // diagnostics (SVTGPU_WR_STATS): thread 0's pass time (candidate start to the first barrier), its control step
    // and the whole descent, in 100 MHz ticks, kept in LDS ({run start, pass, control, mark}: no registers)
    __shared__ unsigned long long s_wt[6];
    __shared__ uint32_t           s_wp[WR_NT / 64]; // each wave's pass time of the current candidate
    if (stat && threadIdx.x == 0)
        s_wt[0] = s_wt[3] = __builtin_amdgcn_s_memrealtime(), s_wt[1] = s_wt[2] = s_wt[4] = s_wt[5] = 0;
    const WrGeo g  = wr_geo(w, h);
    // a wave holds 64 column pairs of one row segment (cpw is a multiple of 64): the segment's values are wave-uniform,
    // which readfirstlane tells the compiler -- the row loop then branches on scalars instead of masking lanes
    const int   cp = threadIdx.x % g.cpw, sg = __builtin_amdgcn_readfirstlane((int)threadIdx.x / g.cpw), x = 2 * cp;
    const int   seg0 = sg * g.R, nrows = __builtin_amdgcn_readfirstlane(sg < g.nseg ? max(0, min(g.R, h - seg0)) : 0);
    const int   xc = min(x, (w - 1) & ~1), hw = h + 6; // an addressable column for lanes right of the unit
    const uint32_t dmask = x >= w ? 0u : x + 1 >= w ? 0xFFFFu : 0xFFFFFFFFu;
    // the lane's source pixels, one (x, x+1) pair per row: registers (LDS mode, <= WR_RMAX rows), else global memory
    const T   *sbase = (const T *)P.src + (size_t)(uy + seg0) * P.sstride + ux + xc;
    const bool s1    = xc + 1 < w; // an odd unit width: the lane's second column is outside the unit
    auto       load_src = [&](int k) -> uint32_t {
        const T *q = sbase + (size_t)k * P.sstride;
        return (uint32_t)q[0] | ((uint32_t)(s1 ? q[1] : 0) << 16);
    };
    uint32_t sv[LDSW ? WR_RMAX : 1];
    if constexpr (LDSW) {
#pragma unroll
        for (int k = 0; k < WR_RMAX; k++)
            if (k < nrows) sv[k] = load_src(k);
    }
    const WienerRound rr  = wiener_round(P.bd);
    const int         lim = (1 << (P.bd + 1 + 7 - rr.r0)) - 1, maxv = (1 << P.bd) - 1;
    const int         hb = (1 << (P.bd + 6)) + (1 << (rr.r0 - 1)), vb = (1 << (rr.r1 - 1)) - (1 << (P.bd + rr.r1 - 1));
    const int         jend = ((nrows + 1) >> 1) + 3;
    int               rounds = 0;
    // one candidate over the lane's rows: its error sum.  Taps uniform (scalar registers), the add-source 128 folded
    // into the centre taps
    auto eval = [&](const int *tap_h, const int *tap_v) -> int {
        // the row bounds made opaque per candidate: the unrolled steps' conditions then stay scalar compares, where
        // the compiler otherwise hoisted all of them out of the candidate loop as 64-bit lane masks and spilled them
        int je = jend, nr = nrows;
        asm volatile("" : "+s"(je), "+s"(nr));
        int hf[8], vf[8];
#pragma unroll
        for (int k = 0; k < 8; k++) hf[k] = tap_h[k], vf[k] = tap_v[k];
        hf[3] += 128, vf[3] += 128;
        auto sp = [](int lo, int hi) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)pack2(lo, hi)); };
        const uint32_t He0 = sp(0, hf[0]), He1 = sp(hf[1], hf[2]), He2 = sp(hf[3], hf[4]), He3 = sp(hf[5], hf[6]);
        const uint32_t Ho0 = sp(hf[0], hf[1]), Ho1 = sp(hf[2], hf[3]), Ho2 = sp(hf[4], hf[5]), Ho3 = sp(hf[6], 0);
        const uint32_t Ve0 = sp(vf[0], vf[1]), Ve1 = sp(vf[2], vf[3]), Ve2 = sp(vf[4], vf[5]), Ve3 = sp(vf[6], 0);
        const uint32_t Vo0 = sp(0, vf[0]), Vo1 = sp(vf[1], vf[2]), Vo2 = sp(vf[3], vf[4]), Vo3 = sp(vf[5], vf[6]);
        auto hclip = [&](int s) { return clamp0_s(s >> rr.r0, lim); };
        auto vclip = [&](int s) { return clamp0_s(s >> rr.r1, maxv); };
        uint32_t hq0[4] = {0, 0, 0, 0}, hq1[4] = {0, 0, 0, 0}; // vertical pairs of the horizontal pass, x and x+1
        uint32_t pa[5], pb[5], na[5], nb[5];
        int      e = 0; // <= 2 * 77 squared errors of <= 1023^2
        // step j: the horizontal pass of window rows seg0+2j, +1 (unit rows seg0+2j-3, -2) at columns x, x+1 (pa, pb);
        // from j = 3 on, output rows seg0+2i, +1 (i = j-3) from horizontal rows 2i-3 .. 2i+4 against source pairs sa, sb
        auto step = [&](int j, uint32_t sa, uint32_t sb) {
            const int a0 = hclip(dot2(pa[3], He3, dot2(pa[2], He2, dot2(pa[1], He1, dot2_s(pa[0], He0, hb)))));
            const int b0 = hclip(dot2(pa[4], Ho3, dot2(pa[3], Ho2, dot2(pa[2], Ho1, dot2_s(pa[1], Ho0, hb)))));
            const int a1 = hclip(dot2(pb[3], He3, dot2(pb[2], He2, dot2(pb[1], He1, dot2_s(pb[0], He0, hb)))));
            const int b1 = hclip(dot2(pb[4], Ho3, dot2(pb[3], Ho2, dot2(pb[2], Ho1, dot2_s(pb[1], Ho0, hb)))));
            hq0[0] = hq0[1], hq0[1] = hq0[2], hq0[2] = hq0[3], hq0[3] = pack2(a0, a1);
            hq1[0] = hq1[1], hq1[1] = hq1[2], hq1[2] = hq1[3], hq1[3] = pack2(b0, b1);
            if (j >= 3) {
                const int i  = j - 3;
                const int o0 = vclip(dot2(hq0[3], Ve3, dot2(hq0[2], Ve2, dot2(hq0[1], Ve1, dot2_s(hq0[0], Ve0, vb)))));
                const int o1 = vclip(dot2(hq1[3], Ve3, dot2(hq1[2], Ve2, dot2(hq1[1], Ve1, dot2_s(hq1[0], Ve0, vb)))));
                const uint32_t d0 = (uint32_t)__builtin_bit_cast(int, __builtin_bit_cast(v2i16, pack2(o0, o1)) -
                                                                          __builtin_bit_cast(v2i16, sa)) & dmask;
                e = dot2(d0, d0, e);
                if (2 * i + 1 < nr) {
                    const int q0 = vclip(dot2(hq0[3], Vo3, dot2(hq0[2], Vo2, dot2(hq0[1], Vo1, dot2_s(hq0[0], Vo0, vb)))));
                    const int q1 = vclip(dot2(hq1[3], Vo3, dot2(hq1[2], Vo2, dot2(hq1[1], Vo1, dot2_s(hq1[0], Vo0, vb)))));
                    const uint32_t d1 = (uint32_t)__builtin_bit_cast(int, __builtin_bit_cast(v2i16, pack2(q0, q1)) -
                                                                              __builtin_bit_cast(v2i16, sb)) & dmask;
                    e = dot2(d1, d1, e);
                }
            }
        };
        if (nr) {
            wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0, na);
            wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0 + 1, nb);
        }
        if constexpr (LDSW) { // unrolled: the source pairs are addressed by constants
#pragma unroll
            for (int j = 0; j < WR_RMAX / 2 + 3; j++) {
                if (j < je) { // uniform per wave (one segment per wave)
#pragma unroll
                    for (int k = 0; k < 5; k++) pa[k] = na[k], pb[k] = nb[k];
                    if (j + 1 < je) { // the next pair of window rows is in flight during this step
                        wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0 + 2 * j + 2, na);
                        wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0 + 2 * j + 3, nb);
                    }
                    step(j, j >= 3 ? sv[2 * j - 6] : 0u, j >= 3 ? sv[2 * j - 5] : 0u);
                }
            }
        } else { // window and source rows from global memory, one step ahead
            uint32_t sa = 0, sb = 0;
#pragma unroll 1
            for (int j = 0; j < je; j++) {
#pragma unroll
                for (int k = 0; k < 5; k++) pa[k] = na[k], pb[k] = nb[k];
                const uint32_t ca = sa, cb = sb;
                if (j + 1 < je) {
                    wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0 + 2 * j + 2, na);
                    wr_fetch<T, LDSW>(win, ws, P, ux, uy, hw, xc, seg0 + 2 * j + 3, nb);
                }
                const int in = j - 2; // the output pair of the next step
                if (in >= 0 && 2 * in < nr) sa = load_src(2 * in), sb = 2 * in + 1 < nr ? load_src(2 * in + 1) : 0u;
                step(j, ca, cb);
            }
        }
        return e;
    };
    // Self-stepping (one-part units, default): every wave holds the descent in its own scalar registers and steps it
    // from the candidate's SSE -- one barrier per candidate, no wave waits on thread 0's step through LDS (which cost
    // ~1.1 of the ~9 us per candidate).  SVTGPU_WR_CLASSIC=1 keeps thread 0's step (the row-part units always do:
    // their SSE exchange runs on one thread)
    if (it.nparts == 1 && !classic) {
        __shared__ unsigned long long s_part2[2][WR_NT / 64];
        Descent Dw   = uniform(D);
        bool    live = __builtin_amdgcn_readfirstlane(*s_mode) != 0;
        while (live) {
            int tv[3], th[8], tvv[8];
            Dw.taps(0, tv);
            th[0] = th[6] = tv[0], th[1] = th[5] = tv[1], th[2] = th[4] = tv[2], th[3] = -2 * (tv[0] + tv[1] + tv[2]), th[7] = 0;
            Dw.taps(1, tv);
            tvv[0] = tvv[6] = tv[0], tvv[1] = tvv[5] = tv[1], tvv[2] = tvv[4] = tv[2], tvv[3] = -2 * (tv[0] + tv[1] + tv[2]);
            tvv[7] = 0;
            const int e = eval(th, tvv);
            const unsigned long long et = wave_sum_u32_wide((uint32_t)e);
            if ((threadIdx.x & 63) == WAVE_LAST) s_part2[rounds & 1][threadIdx.x >> 6] = et;
            if (stat && threadIdx.x == 0) s_wt[1] += __builtin_amdgcn_s_memrealtime() - s_wt[3];
            __syncthreads();
            unsigned long long err = 0;
#pragma unroll
            for (int k = 0; k < WR_NT / 64; k++) err += s_part2[rounds & 1][k];
            npx += (unsigned long long)w * h;
            ++rounds;
            const bool ok = rounds <= WR_MAX_ROUNDS; // a descent always ends: an internal failure, reported by the host
            if (!ok && threadIdx.x == 0) atomicOr(status, 1);
            if (ok) Dw.report(readlane64((long long)err, 0));
            live = ok && Dw.next();
            if (stat && threadIdx.x == 0) s_wt[3] = __builtin_amdgcn_s_memrealtime();
        }
        if (threadIdx.x == 0) D = Dw;
    } else
    while (*s_mode) {
        int e;
        {
            int th[8], tvv[8];
#pragma unroll
            for (int k = 0; k < 8; k++) th[k] = s_taps[k], tvv[k] = s_taps[8 + k];
            e = eval(th, tvv);
        }
        // the unit's SSE, then lane 0's descent step
        const unsigned long long et = wave_sum_u32_wide((uint32_t)e);
        if ((threadIdx.x & 63) == WAVE_LAST) s_part[threadIdx.x >> 6] = et;
        if (stat && (threadIdx.x & 63) == 0) s_wp[threadIdx.x >> 6] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - s_wt[3]);
        if (stat && threadIdx.x == 0) s_wt[1] += __builtin_amdgcn_s_memrealtime() - s_wt[3];
        __syncthreads();
        if (stat && threadIdx.x == 0) {
            uint32_t mx = 0, mn = ~0u;
            for (int q = 0; q < WR_NT / 64; q++) mx = max(mx, s_wp[q]), mn = min(mn, s_wp[q]);
            s_wt[4] += mx, s_wt[5] += mn;
            s_wt[3] = __builtin_amdgcn_s_memrealtime();
        }
        if (threadIdx.x == 0) {
            // the descent step is the unit's serial critical path: its wave issues ahead of the other workgroups'
            // pixel waves on this SIMD while it runs
            __builtin_amdgcn_s_setprio(3);
            unsigned long long err = 0;
            for (int k = 0; k < WR_NT / 64; k++) err += s_part[k];
            npx += (unsigned long long)w * h;
            ++rounds;
            bool ok = rounds <= WR_MAX_ROUNDS; // a descent always ends: an internal failure, reported by the host
            if (!ok) atomicOr(status, 1);
            if (ok && it.nparts > 1) { // publish this part's SSE, add the other parts' SSEs of the same round
                const unsigned long long tag = (unsigned long long)(rounds & 0xFFFF) << 48, low = (1ull << 48) - 1;
                __hip_atomic_store(xch + 2 * (it.first + it.part) + (rounds & 1), tag | err, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                for (int q = 0; q < it.nparts && ok; q++) {
                    if (q == it.part) continue;
                    for (unsigned spin = 0;; spin++) {
                        const unsigned long long v = __hip_atomic_load(xch + 2 * (it.first + q) + (rounds & 1),
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((v & ~low) == tag) {
                            err += v & low;
                            break;
                        }
                        if (spin > (1u << 24)) { // ~seconds: never wait forever
                            atomicOr(status, 2);
                            ok = false;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
            if (ok) D.report((int64_t)err);
            *s_mode = 0;
            if (ok && D.next()) {
                int v[3];
                D.taps(0, v), set_wiener_taps(s_taps, v); // f = 0: hfilter, f = 1: vfilter
                D.taps(1, v), set_wiener_taps(s_taps + 8, v);
                *s_mode = 1;
            }
            __builtin_amdgcn_s_setprio(0);
        }
        if (stat && threadIdx.x == 0) s_wt[2] += __builtin_amdgcn_s_memrealtime() - s_wt[3];
        __syncthreads();
        if (stat && threadIdx.x == 0) s_wt[3] = __builtin_amdgcn_s_memrealtime();
    }
    if (stat && threadIdx.x == 0) {
        atomicAdd(stat + 0, 1ull), atomicAdd(stat + 1, (unsigned long long)rounds);
        atomicAdd(stat + 2, __builtin_amdgcn_s_memrealtime() - s_wt[0]), atomicAdd(stat + 3, s_wt[2]);
        atomicAdd(stat + 4, s_wt[1]), atomicAdd(stat + 5, (unsigned long long)w * h);
        atomicAdd(stat + 6, (unsigned long long)(it.nparts > 1)), atomicAdd(stat + 7, s_wt[4]);
        atomicAdd(stat + 8, s_wt[5]);
    }
}

template <typename T>
__global__ __launch_bounds__(WR_NT) void wiener_res_kernel(const SearchArgs A, Descent *ds, const WrItem *items,
                                                           int lds_cap, unsigned long long *xch, int32_t *status,
                                                           unsigned long long *pc, unsigned long long *stat,
                                                           unsigned long long *tk, int classic) {
    PROF_BEGIN(tk);
    extern __shared__ uint32_t wr_win[]; // the part's CDEF window (LDS mode)
    __shared__ uint64_t           s_draw[sizeof(Descent) / 8];
    __shared__ unsigned long long s_part[WR_NT / 64];
    __shared__ int16_t            s_taps[16];
    __shared__ int                s_mode;
    Descent         &D  = *(Descent *)s_draw;
    const WrItem     it = items[blockIdx.x];
    const int        u  = it.unit;
    const URect      ur = A.units[u];
    const PlaneArgs &P  = A.pl[A.tiles[A.tile0[u]].plane];
    const int        ux = ur.h_start, uy = ur.v_start + it.y0, w = ur.h_end - ur.h_start, h = it.y1 - it.y0;
    const int        ws = (w + 10) >> 1;
    const bool       lds = wr_lds_mode(w, h, lds_cap);
    if (threadIdx.x == 0) {
        D      = ds[u];
        s_mode = 0;
        if (!D.done && D.next()) {
            int v[3];
            D.taps(0, v), set_wiener_taps(s_taps, v);
            D.taps(1, v), set_wiener_taps(s_taps + 8, v);
            s_mode = 1;
        }
    }
    if (lds) { // stage the edge-clamped window: rows uy-3 .., columns ux-4 .. (pairs)
        const T *d = (const T *)P.dgd;
        for (int i = threadIdx.x; i < (h + 6) * ws; i += WR_NT) {
            const int r = i / ws, c = 2 * (i - r * ws);
            const int fy = min(max(uy - 3 + r, 0), P.H - 1), f0 = min(max(ux - 4 + c, 0), P.W - 1),
                      f1 = min(max(ux - 3 + c, 0), P.W - 1);
            const T *row = d + (size_t)fy * P.dstride;
            wr_win[i]    = (uint32_t)row[f0] | ((uint32_t)row[f1] << 16);
        }
    }
    __syncthreads();
    unsigned long long npx = 0;
    if (lds) wr_run<T, true>(A, P, D, wr_win, ws, ux, uy, w, h, it, xch, &s_mode, s_taps, s_part, status, npx, stat, classic != 0);
    else wr_run<T, false>(A, P, D, wr_win, ws, ux, uy, w, h, it, xch, &s_mode, s_taps, s_part, status, npx, stat, classic != 0);
    if (threadIdx.x == 0 && it.part == 0) ds[u] = D;
    if (pc && threadIdx.x == 0 && npx) atomicAdd(pc + (blockIdx.x & (PROF_SP - 1)), npx);
    PROF_END(tk);
}

// svt_decode_xq (EbRestoration.c:634-646): xq of the ep's absent filter is 0
__device__ inline void decode_xq(const Descent &d, int32_t *xq) {
    const int x0 = d.val(0, 0), x1 = d.val(0, 1), r0 = c_sgr_r[d.ep][0], r1 = c_sgr_r[d.ep][1];
    xq[0] = r0 == 0 ? 0 : x0;
    xq[1] = r0 == 0 ? 128 - x1 : r1 == 0 ? 0 : 128 - x0 - x1;
}

// Self-guided descents evaluate a speculative tree per pass: node 0 is the pending candidate, node n's children
// 2n+1 / 2n+2 are the candidates proposed after a worse / not-worse outcome of node n.  The walk replays the
// outcomes against the measured errors (report() decides exactly as the reference does) and stops at the first
// candidate that was not evaluated, which becomes the next root.
// the speculative tree of depth_nodes nodes below d's pending candidate: node n's xq pair at cd[2n], the mask of the
// nodes built (tree: SG_NC / 2 nodes of scratch)
__device__ uint32_t sgr_tree(const Descent &d, int depth_nodes, int32_t *cd, Descent *tree) {
    uint32_t mask = 1;
    decode_xq(d, cd);
    tree[0] = d;
    for (int nd = 0; nd < SG_NC / 2; nd++) {
        if (!(mask >> nd & 1) || 2 * nd + 1 >= depth_nodes) continue;
        for (int w = 1; w >= 0; w--) {
            if (w && tree[nd].init) continue; // the seed's outcome does not steer the descent
            Descent c = tree[nd];
            c.report_outcome(w != 0, 0);
            if (!c.next()) continue;
            const int ch = 2 * nd + (w ? 1 : 2);
            decode_xq(c, cd + 2 * ch);
            mask |= 1u << ch;
            if (ch < SG_NC / 2) tree[ch] = c;
        }
    }
    return mask;
}

// the descent's steps through an evaluated tree (errors by node): exactly the reference's decisions, stopping at the
// first candidate that was not evaluated (the next root) or at the end of the descent
template <typename ErrAt>
__device__ void sgr_replay(Descent &d, uint32_t evaluated, ErrAt &&err_at) {
    for (int node = 0;;) {
        const int64_t v     = err_at(node);
        const bool    worse = !d.init && v > d.err;
        d.report(v);
        if (!d.next()) break;
        node = 2 * node + (worse ? 1 : 2);
        if (node >= SG_NC || !(evaluated >> node & 1)) break;
    }
}

// the plane of global unit u
__device__ inline int unit_plane(const SearchArgs &A, int nplanes, int u) {
    int p = 0;
    while (p + 1 < nplanes && u >= A.pl[p + 1].unit_base) p++;
    return p;
}

// ---------------------------------------------------------------------------------------------
// descent seeds on the device
// ---------------------------------------------------------------------------------------------
struct SeedCfg {
    int32_t wn_use_refinement, wn_max_one_step, sg_refine[2];
};


// wiener_decompose_sep_sym + finalize + compute_score (EbRestorationPick.c:906-1040, 1337-1419), one workgroup
// per unit; the unit's descent starts from the finalized taps unless the score says the filter does not help
__global__ __launch_bounds__(256) void wiener_solve_kernel(const SearchArgs A, int nplanes, const int64_t *mh,
                                                           const SeedCfg cfg, Descent *ds, SvtGpuRestUnit *wu,
                                                           unsigned long long *tk) {
    PROF_BEGIN(tk);
    __shared__ WienerSolveLds L;
    const int        u = blockIdx.x, tid = threadIdx.x;
    const PlaneArgs &P = A.pl[unit_plane(A, nplanes, u)];
    const int        win = P.win, win2 = win * win, div = P.bd == 10 ? 4 : 1;
    const int64_t   *blk = mh + P.mh_off + (size_t)(u - P.unit_base) * P.nval;
    // assemble M[k] (k = col * win + row) and the full H from the column-pair blocks
    for (int t = tid; t < win2 * win2; t += blockDim.x) {
        const int k = t / win2, l = t % win2, ck = k / win, rk = k % win, cl = l / win, rl = l % win;
        const int c1 = min(ck, cl), c2 = max(ck, cl), r1 = ck <= cl ? rk : rl, r2 = ck <= cl ? rl : rk;
        const int pair = c1 * win - c1 * (c1 - 1) / 2 + (c2 - c1);
        L.H[t] = blk[pair * 49 + r1 * 7 + r2] / div;
    }
    const int npair = win * (win + 1) / 2;
    if (tid < win2) L.M[tid] = blk[npair * 49 + (tid / win) * 7 + tid % win] / div;
    if (tid < win) { // start from the mid taps (centre incl. the implicit step)
        const int init[7] = {3, -7, 15, 128 - 2 * (3 - 7 + 15), 15, -7, 3}, poff = (7 - win) >> 1;
        L.a[tid] = L.b[tid] = (int32_t)(TAP_SCALE / FILT_STEP * init[tid + poff]);
    }
    __syncthreads();
    for (int it = 1; it < 5; it++) {
        update_sep_sym(false, win, L);
        update_sep_sym(true, win, L);
    }
    __shared__ SvtGpuRestUnit w;
    if (tid == 0) {
        for (int k = 0; k < 8; k++) w.vfilter[k] = w.hfilter[k] = 0;
        w.type = SVTGPU_RESTORE_WIENER, w.ep = 0, w.xqd[0] = w.xqd[1] = 0;
        finalize_sym_filter(win, L.a, w.vfilter);
        finalize_sym_filter(win, L.b, w.hfilter);
    }
    __syncthreads();
    const int64_t score = compute_score(win, L, w.vfilter, w.hfilter);
    if (tid == 0) {
        Descent d;
        d.unit = u;
        if (score > 0) { // the unit keeps sse = INT64_MAX
            w.type = 0;
            d.done = true;
        } else {
            d.start = 4;
            d.end   = cfg.wn_use_refinement ? (cfg.wn_max_one_step ? 4 : 1) : 8; // 8: no refinement
            d.cont  = !cfg.wn_max_one_step;
            d.nf = 2, d.p_lo = (7 - win) >> 1, d.p_hi = 2;
            for (int t = 0; t < 3; t++) {
                d.set_bounds(t, c_tap_min[t], c_tap_max[t]);
                d.set_val(0, t, w.hfilter[t]); // f = 0: hfilter, f = 1: vfilter (the reference's order)
                d.set_val(1, t, w.vfilter[t]);
            }
            d.begin();
        }
        ds[u] = d;
        wu[u] = w;
    }
    PROF_END(tk);
}

// svt_get_proj_subspace_c (:417-500) from the exact integer moments, encode_xq (:502-518), and the descent of
// finer_search_pixel_proj_error (:320-413) seeded there; one lane per (unit, ep)
// pair i (plane p) from its moments m[5] = {Σg1², Σg2², Σg1g2, Σg1·s, Σg2·s}: the seeded descent
__device__ Descent sgr_seed(const SearchArgs &A, int p, int i, const int64_t *m, const SeedCfg &cfg) {
    const PlaneArgs &P  = A.pl[p];
    const int        ul = (i - P.pair_base) / P.ne, k = (i - P.pair_base) % P.ne, ep = P.eps[k];
    const URect      ur = A.units[P.unit_base + ul];
    const double     size = (double)((ur.h_end - ur.h_start) * (ur.v_end - ur.v_start));
    double H00 = (double)m[0], H11 = (double)m[1], H01 = (double)m[2], C0 = (double)m[3], C1 = (double)m[4];
    H00 /= size, H01 /= size, H11 /= size;
    const double H10 = H01;
    C0 /= size, C1 /= size;
    const int r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
    int32_t   xq[2] = {0, 0};
    if (r0 == 0) {
        if (!(H11 < 1e-8)) xq[1] = (int32_t)rint(C1 / H11 * (1 << 7));
    } else if (r1 == 0) {
        if (!(H00 < 1e-8)) xq[0] = (int32_t)rint(C0 / H00 * (1 << 7));
    } else {
        const double det = H00 * H11 - H01 * H10;
        if (!(det < 1e-8)) {
            xq[0] = (int32_t)rint((H11 * C0 - H01 * C1) / det * (1 << 7));
            xq[1] = (int32_t)rint((H00 * C1 - H10 * C0) / det * (1 << 7));
        }
    }
    int xd0, xd1;
    if (r0 == 0) {
        xd0 = 0;
        xd1 = min(max(128 - xq[1], PRJ_MIN1), PRJ_MAX1);
    } else if (r1 == 0) {
        xd0 = min(max(xq[0], PRJ_MIN0), PRJ_MAX0);
        xd1 = min(max(128 - xd0, PRJ_MIN1), PRJ_MAX1);
    } else {
        xd0 = min(max(xq[0], PRJ_MIN0), PRJ_MAX0);
        xd1 = min(max(128 - xd0 - xq[1], PRJ_MIN1), PRJ_MAX1);
    }
    Descent d;
    d.unit = P.unit_base + ul, d.k = k, d.ep = ep;
    d.start = 2, d.end = cfg.sg_refine[p > 0] ? 1 : 4, d.cont = true, d.nf = 1, d.p_lo = 0, d.p_hi = 1;
    d.set_bounds(0, PRJ_MIN0, PRJ_MAX0), d.set_bounds(1, PRJ_MIN1, PRJ_MAX1);
    d.skipm = (r0 == 0 ? 1u : 0u) | (r1 == 0 ? 2u : 0u);
    d.set_val(0, 0, xd0), d.set_val(0, 1, xd1);
    d.begin();
    return d;
}

// best ep per unit (strict <, first) -> best[unit] = {ep index, ep, xq0, xq1}, raw[unit] = the descent's two values
// (what the host's records hold: only these come back, not every (unit, ep) descent)
__global__ void sgr_best_kernel(const Descent *ds, const SearchArgs A, int nplanes, int n, int32_t *best, int32_t *raw) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    int p = 0;
    while (p + 1 < nplanes && u >= A.pl[p + 1].unit_base) p++;
    const PlaneArgs &P    = A.pl[p];
    const Descent   *d    = ds + P.pair_base + (u - P.unit_base) * P.ne;
    long long        be   = -1;
    int              bk   = 0;
    for (int k = 0; k < P.ne; k++)
        if (be == -1 || d[k].err < be) be = d[k].err, bk = k;
    const int ep = P.eps[bk], x0 = d[bk].val(0, 0), x1 = d[bk].val(0, 1);
    best[4 * u]     = bk;
    best[4 * u + 1] = ep;
    best[4 * u + 2] = c_sgr_r[ep][0] == 0 ? 0 : x0;
    best[4 * u + 3] = c_sgr_r[ep][0] == 0 ? 128 - x1 : c_sgr_r[ep][1] == 0 ? 0 : 128 - x0 - x1;
    raw[2 * u] = x0, raw[2 * u + 1] = x1;
}

// ---------------------------------------------------------------------------------------------
// The self-guided search of one (unit, ep) per workgroup with the unit resident on the CU (default).
// search_selfguided_restoration (EbRestorationPick.c:550-652) per ep: the projection subspace from the filtered unit
// (svt_get_proj_subspace, :417-500), encode_xq, then finer_search_pixel_proj_error's descent (:320-411), every
// candidate a pass over all the unit's pixels.  The filter planes of the ep (sgr_flt_kernel) are read exactly once.
// A workgroup is 15 pixel waves and one control wave:
//   * pixel lane l (0..959) owns 4-pixel chunks l, l + 960, ... of the unit (row-major over 4-pixel columns), at most
//     SR_KMAX of them: g = (flt0 - u, flt1 - u) packed int16 per pixel in registers (72 VGPRs), the (x - src) pairs
//     in LDS (135 KB); chunks past the unit hold zeros, which add nothing to any sum.  The pixel waves form the five
//     projection moments (exact 64-bit sums) while loading, and per pass the errors of the
//     pending candidates -- per pixel and candidate one v_dot2 with the rounding and (x - src) * 2^11 terms in its
//     accumulator, a shift, a multiply-add;
//   * the control wave holds the descent in registers and steps it between the passes, lane-parallel: lane c sums
//     candidate c's wave partials (and exchanges it with the other row parts), every lane replays the evaluated tree
//     (sgr_replay: the reference's decisions), and lane n builds node n of the next speculative tree by applying the
//     outcomes on its path to the root (the per-round path's sgr_tree, one node per lane); lane 0 seeds the descent
//     from the moments (sgr_seed: the reference's double arithmetic).  Two workgroup barriers per pass, nothing in
//     global memory, and the pixel waves' registers are never live in the control code;
//   * units larger than SR_MAX_PX (the frame's bottom luma unit row, 256 x 376 at 4K) are cut into row parts on
//     workgroups adjacent in their XCD's dispatch order; their moments and candidate errors meet through uncached
//     memory each pass (tagged 64-bit words, double-buffered by pass parity, bounded waits), every part taking the
//     same steps.
// The pass count is bounded (SR_MAX_PASSES; a descent ends far earlier): on overflow or a timed-out exchange the
// descent stops and *status is set, which search_frame reports as SVTGPU_ERR_HIP.
// ---------------------------------------------------------------------------------------------
// Two 512-lane workgroups per CU (7 pixel waves + 1 control wave each, 68 KB of LDS): one workgroup's loads, control
// steps and barriers overlap the other's passes (1024-lane workgroups, one per CU: 2204 vs 2366 Mpx/s at three frames
// in flight, 1656 vs 1740 at one, same box, profiles/r03/srvar)
#ifndef SVTGPU_SR_GLDS
#define SVTGPU_SR_GLDS 0 // 1: the load phase's dx chunks by direct global -> LDS loads (A/B)
#endif
#ifndef SVTGPU_SR_NT
#define SVTGPU_SR_NT 512
#endif
#ifndef SVTGPU_SR_KMAX
#define SVTGPU_SR_KMAX 19 // resident 4-pixel chunks per pixel lane: parts of <= 34048 pixels (256 x 133 luma)
#endif
constexpr int SR_NT = SVTGPU_SR_NT, SR_PW = SR_NT / 64 - 1, SR_PL = SR_PW * 64, SR_KMAX = SVTGPU_SR_KMAX;
constexpr int SR_LB = 4; // chunks whose loads are in flight together in the load phase
constexpr int SR_MAX_PX = SR_PL * SR_KMAX * 4;
constexpr int SR_MAX_PASSES = 4096, SR_MAX_PARTS = 8;
constexpr int SR_LDS = SR_KMAX * SR_PL * 8; // the (x - src) pairs of the part
struct SrItem {
    int32_t pair, y0, y1, part, nparts, first; // rows [y0, y1) of the pair's unit; part q at grid position first + 8 q
};
constexpr unsigned long long SR_LOW = (1ull << 48) - 1;

// one lane's value of exchange round r, summed over the row parts (this part's value published first).  Every value
// fits 48 bits two's complement: a part holds <= 2^17 pixels, g in [-16368, 32767], |s| < 2^14, and a projection
// error |e| <= (352 * 32767 + 2^21) / 2^11 < 6657 (|xq0| <= 96, |xq1| <= 256), e^2 < 2^26.  false: timed out
// xmode bit 9: one-part items keep the two-barrier pass loop (A/B).  Bit 8: the words live in cached memory and stay in the XCD's L2 (every part of an item runs on one XCD: grid
// positions first + 8 q); the store is a plain one (the CU's L1 writes through to the L2), the polls bypass the L1
// (agent-scope loads).  Bits 0-7: the search's epoch, in the tag with the exchange round, so that a line an earlier
// search left in an L2 never passes for this one's.  xmode 0: uncached memory, agent-scope stores.
__device__ bool sr_exchange_lane(unsigned long long *xch, const SrItem &it, int r, int q, long long &v,
                                 int32_t *status, unsigned xmode) {
    const unsigned long long tag = (unsigned long long)(((xmode & 0xFF) << 8) | ((r + 1) & 0xFF)) << 48;
    unsigned long long *mine = xch + ((size_t)(it.first + 8 * it.part) * 2 + (r & 1)) * 8 + q;
    const unsigned long long word = tag | ((unsigned long long)v & SR_LOW);
    if (xmode & 0x100)
        __hip_atomic_store(mine, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        __hip_atomic_store(mine, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long add = 0;
    for (int p = 0; p < it.nparts; p++) {
        if (p == it.part) continue;
        const unsigned long long *o = xch + ((size_t)(it.first + 8 * p) * 2 + (r & 1)) * 8 + q;
        for (unsigned spin = 0;; spin++) {
            const unsigned long long w = __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((w & ~SR_LOW) == tag) {
                add += (long long)(w << 16) >> 16;
                break;
            }
            if (spin > (1u << 24)) { // ~seconds: never wait forever
                atomicOr(status, 2);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    v += add;
    return true;
}

// control wave: node n (= this lane) of the speculative tree below d's pending candidate -- the root's state with the
// outcomes on the path to n applied (children of m: 2m + 1 after a worse outcome, 2m + 2 otherwise); nodes exist up
// to SG_NC, a node's children only below SG_NC / 2, and the seed's outcome does not steer the descent.  The tree's
// candidates go to s_xq compacted in node order, the node mask to *s_mask, the count to *s_nv (0: the descent ended)
__device__ __forceinline__ void sr_tree_lanes(const Descent &d, bool live, int nodes, uint32_t *s_xq, uint32_t *s_mask,
                                              int *s_nv) {
    const int n  = threadIdx.x & 63;
    bool      ok = live && n < nodes; // nodes: 1, 3 or SG_NC (a complete tree)
    uint32_t  xv = 0;
    if (ok) {
        int path = 0, depth = 0; // outcome bits from the node up to the root
        for (int m = n; m > 0; m = (m - 1) >> 1) path |= (m & 1) << depth++;
        Descent c = d;
        for (int i = depth - 1; i >= 0 && ok; i--) {
            const bool worse = path >> i & 1;
            if (worse && c.init) ok = false;
            else {
                c.report_outcome(worse, 0);
                ok = c.next();
            }
        }
        int32_t x[2];
        decode_xq(c, x);
        xv = pack2(x[0], x[1]);
    }
    const unsigned long long mask = __ballot(ok);
    if (ok) s_xq[__popcll(mask & ((1ull << n) - 1))] = xv;
    if (n == 0) *s_mask = (uint32_t)mask, *s_nv = (int)__popcll(mask);
}

// control wave, one-candidate passes: the two candidates that can follow d's pending one -- after a worse outcome and
// after a not-worse one (the seed's outcome does not steer: no worse child) -- built while the pixel waves evaluate the
// pending candidate, so that after its error only the choice between them is left before the next pass.  d is
// wave-uniform, so both children are built one after the other in scalar registers (the scalar unit, no divergent
// lanes: two lanes each stepping one child ran both paths on the vector unit, as long as the pixel pass itself).
// (ok*, x*) wave-uniform; !ok: the descent ends on that outcome.
__device__ __forceinline__ void sr_children(const Descent &d, uint32_t &xw, bool &okw, uint32_t &xb, bool &okb) {
    okw = false, xw = 0;
    if (!d.init) {
        Descent c = d;
        c.report_outcome(true, 0);
        okw = c.next();
        if (okw) {
            int32_t x[2];
            decode_xq(c, x);
            xw = pack2(x[0], x[1]);
        }
    }
    Descent c = d;
    c.report_outcome(false, 0);
    okb = c.next();
    xb  = 0;
    if (okb) {
        int32_t x[2];
        decode_xq(c, x);
        xb = pack2(x[0], x[1]);
    }
}

// the next tree: a single node (the pending candidate itself) from the uniform descent, else one node per lane
__device__ __forceinline__ void sr_tree_publish(const Descent &d, bool live, int nodes, uint32_t *s_xq,
                                                uint32_t *s_mask, int *s_nv) {
    if (nodes == 1) {
        if ((threadIdx.x & 63) == 0) {
            int32_t x[2];
            decode_xq(d, x);
            s_xq[0] = pack2(x[0], x[1]);
            *s_mask = 1, *s_nv = live ? 1 : 0;
        }
    } else {
        sr_tree_lanes(d, live, nodes, s_xq, s_mask, s_nv);
    }
}

// one pass over the resident pixels: the errors of the first nv (<= NV) candidates, wave totals into s_red[wave].
// Candidates past nv are evaluated with xq = 0 and dropped (NV = nv up to 4; 7 for trees of 5-7 nodes).
// The (x - src) pairs are read from LDS four chunks at a time: one LDS latency per group of four chunks instead of
// one per chunk (the load phase leaves zeros in the chunks from K up to the next multiple of four, so a group never
// needs a per-chunk guard).  Issuing the next group's reads before the current group spills the load phase's registers.
template <int NV>
__device__ __forceinline__ void sr_pass(const uint32_t (&g)[SR_KMAX][4], const uint32_t *dx, int pl, int K, int nv,
                                        const uint32_t *s_xq, unsigned long long (*s_red)[SG_NC]) {
    static_assert(SR_LB == 4, "the load phase zero-fills whole groups of four chunks");
    constexpr int GS = NV == 1 ? 4 : 1, NG = (SR_KMAX + GS - 1) / GS;
    uint32_t xq[NV], acc[NV];
#pragma unroll
    // the candidates stay in VGPRs: v_dot2_i32_i16 (VOP3) then takes the rounding constant from an SGPR, with no
    // per-pixel copy into an accumulating v_dot2c
    for (int c = 0; c < NV; c++) xq[c] = c < nv ? s_xq[c] : 0u, acc[c] = 0;
#pragma unroll
    for (int gi = 0; gi < NG; gi++) {
        const int kb = GS * gi;
        if (kb < K) { // uniform: the group's reads issued together
            uint2 cur[GS];
#pragma unroll
            for (int j = 0; j < GS; j++)
                if (kb + j < SR_KMAX) cur[j] = make_uint2(dx[(kb + j) * SR_PL + pl], dx[(SR_KMAX + kb + j) * SR_PL + pl]);
#pragma unroll
            for (int j = 0; j < GS; j++) {
                const int kk = kb + j;
                if (kk >= SR_KMAX) break;
                const uint2 dw = cur[j];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t w  = q < 2 ? dw.x : dw.y;
                    // floor((v + 1024) / 2^11) + (x - src): the int16 half is added as an SDWA operand (no extraction)
                    const int      d1 = (q & 1) ? (int)(int16_t)(w >> 16) : (int)(int16_t)w;
#pragma unroll
                    for (int c = 0; c < NV; c++) {
                        const int ee = (dot2_s(g[kk][q], xq[c], 1024) >> 11) + d1;
                        acc[c] += (uint32_t)(ee * ee);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NV; c++)
        if (c < nv) {
            const unsigned long long t = wave_sum_u32_wide(acc[c]); // <= 76 e^2 < 2^32 per lane
            if ((pl & 63) == WAVE_LAST) s_red[pl >> 6][c] = t;
        }
}

// TREE: the speculative-tree variants (nodes 3 / 7, several candidates per pass); the default one-candidate kernel
// compiles only sr_pass<1>, which leaves the registers for its grouped LDS reads
template <typename T, bool TREE>
__global__ __launch_bounds__(SR_NT, 4) void sgr_res_kernel(const SearchArgs A, int nplanes, const SrItem *items,
                                                        const SeedCfg cfg, int nodes_arg, Descent *ds,
                                                        unsigned long long *xch, unsigned xmode, int32_t *status,
                                                        unsigned long long *stat, unsigned long long *tk) {
    PROF_BEGIN(tk);
    // one node per pass in the default kernel: a compile-time constant there, so the per-lane tree builder (a
    // divergent Descent copy per lane) is not compiled in and the descent keeps to registers
    const int nodes = TREE ? nodes_arg : 1;
    // [half][chunk k][pixel lane]: (x - src) of pixels 0, 1 (half 0) and 2, 3 (half 1), int16 pairs -- two planes of
    // lane-linear words, the layout the direct global -> LDS loads (SVTGPU_SR_GLDS) write
    extern __shared__ uint32_t sr_dx[];
    // wave partials: the moments, then each pass's errors; two buffers by pass parity (the one-barrier path of
    // one-part items reads a pass's partials while the next pass writes the other buffer)
    __shared__ unsigned long long s_red2[2][SR_PW][SG_NC];
    unsigned long long (*const s_red)[SG_NC] = s_red2[0];
    // one-barrier path: the seeded descent every wave steps itself (raw storage: Descent has member initializers)
    __shared__ __attribute__((aligned(8))) unsigned char s_desc_raw[sizeof(Descent)];
    Descent &s_desc = *reinterpret_cast<Descent *>(s_desc_raw);
    __shared__ unsigned long long s_etot[2]; // self-stepping row parts: each pass's error summed over the parts
    __shared__ int                s_xok[2];  // ... and whether the exchange succeeded
    __shared__ uint32_t           s_xq[SG_NC];         // the pending tree's candidates (xq pairs), compacted
    __shared__ uint32_t           s_mask;              // its nodes
    __shared__ int                s_nv;                // its candidate count (0: the descent has ended)
    const SrItem it = items[blockIdx.x];
    if (it.pair < 0) return; // an empty slot of the XCD-ordered grid (uniform)
    int p = 0;
    while (p + 1 < nplanes && it.pair >= A.pl[p + 1].pair_base) p++;
    const PlaneArgs &P  = A.pl[p];
    const int        ul = (it.pair - P.pair_base) / P.ne, k = it.pair - P.pair_base - ul * P.ne, ep = P.eps[k];
    const URect      ur = A.units[P.unit_base + ul];
    const int        uw = ur.h_end - ur.h_start, cw = (uw + 3) >> 2, nch = cw * (it.y1 - it.y0), K = (nch + SR_PL - 1) / SR_PL;
    if (K > SR_KMAX || nch <= 0) { // the host plans parts of <= SR_MAX_PX pixels; never index past the registers
        if (threadIdx.x == 0) atomicOr(status, 4);
        return;
    }
    // the wave's role from a scalar (readfirstlane) condition: the compiler then treats each role's code as uniform
    // control flow -- with `threadIdx.x < SR_PL` it could not prove the branch wave-uniform and compiled the control
    // wave's descent steps as exec-masked vector code with scratch traffic
    if (__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) < SR_PW) {
        // ================= pixel waves =================
        const int      pl = threadIdx.x, r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
        const T       *d = (const T *)P.dgd, *s = (const T *)P.src;
        const size_t   pn = (size_t)P.fstride * P.H;
        // an ep without one of the filters reads a plane that holds no data: its g half is zeroed
        const int16_t *f0 = P.flt + (size_t)k * 2 * pn, *f1 = P.flt + (size_t)P.f1e[k] * 2 * pn + pn;
        const uint32_t gmask = (r0 ? 0x0000FFFFu : 0u) | (r1 ? 0xFFFF0000u : 0u);
        // ---- load the part: g in registers, (x - src) in LDS, the moments on the way ----
        // Chunk kk of this lane is chunk c = pl + kk * SR_PL of the part (row-major over 4-sample columns); its
        // (row, column) advance by a fixed step from one kk to the next (no division per chunk).  Chunks past the part
        // read the part's last chunk (addresses stay inside) and contribute zeros.
        const int      dr = SR_PL / cw, dc = SR_PL - dr * cw, lastc = nch - 1, lrow = lastc / cw, lcol = lastc - lrow * cw;
        int            crow = pl / cw, ccol = pl - crow * cw; // chunk 0 of this lane
        auto           chunk_at = [&](int kk, int &row, int &col) {   // (row, col) of chunk kk, clamped into the part
            row = crow, col = ccol;
            if (pl + kk * SR_PL >= nch) row = lrow, col = lcol;
        };
        auto           advance = [&]() {
            crow += dr, ccol += dc;
            if (ccol >= cw) ccol -= cw, crow++;
        };
        // 1. the ep's two filter planes of every chunk, straight into g (raw int16 pairs: flt0 of pixels 0, 1 | 2, 3
        //    then flt1 of them): every HBM read of the part in flight at once, one memory round trip per item
        uint32_t g[SR_KMAX][4];
#pragma unroll
        for (int kk = 0; kk < SR_KMAX; kk++) {
            g[kk][0] = g[kk][1] = g[kk][2] = g[kk][3] = 0u;
            if (kk < K) { // uniform
                int row, col;
                chunk_at(kk, row, col);
                const size_t fo = (size_t)(ur.v_start + it.y0 + row) * P.fstride + ur.h_start + 4 * col;
                // an ep without one of the filters (eps 10-15) reads only the other plane (r0 / r1 uniform)
                const uint2  a0 = r0 ? *(const uint2 *)(f0 + fo) : make_uint2(0u, 0u);
                const uint2  a1 = r1 ? *(const uint2 *)(f1 + fo) : make_uint2(0u, 0u);
                g[kk][0] = a0.x, g[kk][1] = a0.y, g[kk][2] = a1.x, g[kk][3] = a1.y;
                advance();
            }
        }
        // 2. dx = dgd - src (the plane unit_sums_kernel writes; the eps of a unit read it through one L2) in groups of
        //    SR_LB chunks: the moments, and the (x - src) pairs to LDS.  g (1.) already holds flt - (dgd << 4), so a
        //    chunk needs two registers here instead of four for the CDEF output and the source: half the round trips
        crow = pl / cw, ccol = pl - crow * cw;
        unsigned long long M0 = 0, M1 = 0, M2 = 0, M3 = 0, M4 = 0; // M2..M4 hold signed sums mod 2^64
#if SVTGPU_SR_GLDS
        // every chunk's dx straight into its LDS words with direct global -> LDS loads (no registers: one round trip
        // for the part), then each lane reads its own words back, masks them and forms the moments
        {
            uint32_t *lw = sr_dx + (pl & ~63); // the wave's lane-linear base: lane l of the wave lands at lw[l + ...]
#pragma unroll
            for (int kk = 0; kk < SR_KMAX; kk++) {
                if (kk >= K) break; // uniform
                int row, col;
                chunk_at(kk, row, col);
                const int16_t *src = P.dxp + (size_t)(ur.v_start + it.y0 + row) * P.fstride + ur.h_start + 4 * col;
                __builtin_amdgcn_global_load_lds((const void *)src,
                                                 (__attribute__((address_space(3))) void *)(lw + kk * SR_PL), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((const void *)(src + 2),
                                                 (__attribute__((address_space(3))) void *)(lw + (SR_KMAX + kk) * SR_PL),
                                                 4, 0, 0);
                advance();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        crow = pl / cw, ccol = pl - crow * cw;
#pragma unroll
        for (int kk = 0; kk < SR_KMAX; kk++) {
            if (kk >= K) { // uniform: zeros up to the next multiple of SR_LB (sr_pass reads whole groups)
                if (kk < ((K + SR_LB - 1) & ~(SR_LB - 1))) sr_dx[kk * SR_PL + pl] = sr_dx[(SR_KMAX + kk) * SR_PL + pl] = 0u;
                continue;
            }
            int row, col;
            chunk_at(kk, row, col);
            const int nin = pl + kk * SR_PL < nch ? min(4, uw - 4 * col) : 0;
            advance();
            const uint32_t mlo = nin >= 2 ? ~0u : nin == 1 ? 0xFFFFu : 0u;
            const uint32_t mhi = nin >= 4 ? ~0u : nin == 3 ? 0xFFFFu : 0u;
            g[kk][0] &= mlo, g[kk][2] &= mlo, g[kk][1] &= mhi, g[kk][3] &= mhi;
            const uint2 x2 = make_uint2(sr_dx[kk * SR_PL + pl] & mlo, sr_dx[(SR_KMAX + kk) * SR_PL + pl] & mhi);
            if (nin < 4) sr_dx[kk * SR_PL + pl] = x2.x, sr_dx[(SR_KMAX + kk) * SR_PL + pl] = x2.y;
            const int      dxq[4] = {(int)(int16_t)(x2.x & 0xFFFF), (int)x2.x >> 16, (int)(int16_t)(x2.y & 0xFFFF),
                                     (int)x2.y >> 16};
            const uint32_t fw[4] = {__builtin_amdgcn_perm(g[kk][2], g[kk][0], 0x05040100u),
                                    __builtin_amdgcn_perm(g[kk][2], g[kk][0], 0x07060302u),
                                    __builtin_amdgcn_perm(g[kk][3], g[kk][1], 0x05040100u),
                                    __builtin_amdgcn_perm(g[kk][3], g[kk][1], 0x07060302u)};
            uint32_t m0 = 0, m1 = 0;
            int      m3 = 0, m4 = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t gq = fw[q] & gmask;
                const int      g1 = (int)(int16_t)(gq & 0xFFFF), g2 = (int)gq >> 16, ss = -(dxq[q] << 4);
                m0 += (uint32_t)(g1 * g1), m1 += (uint32_t)(g2 * g2);
                m3 += g1 * ss, m4 += g2 * ss;
                M2 += (unsigned long long)(long long)(g1 * g2);
                g[kk][q] = gq;
            }
            M0 += m0, M1 += m1, M3 += (unsigned long long)(long long)m3, M4 += (unsigned long long)(long long)m4;
        }
#else
        constexpr int LB2 = SR_LB;
#pragma unroll
        for (int kb = 0; kb < SR_KMAX; kb += LB2) {
            if (kb >= K) { // uniform: zeros up to the next multiple of SR_LB (sr_pass reads whole groups)
                if (kb < ((K + SR_LB - 1) & ~(SR_LB - 1)))
#pragma unroll
                    for (int j = 0; j < LB2; j++)
                        if (kb + j < SR_KMAX) sr_dx[(kb + j) * SR_PL + pl] = sr_dx[(SR_KMAX + kb + j) * SR_PL + pl] = 0u;
                continue;
            }
            uint2 xv[LB2];
            int   nin[LB2]; // the chunk's pixels inside the part: 4, fewer in the last column of a crop width that is
                            // not a multiple of 4, none past the part
#pragma unroll
            for (int j = 0; j < LB2; j++) { // the group's loads in flight together
                xv[j] = make_uint2(0u, 0u), nin[j] = 0;
                if (kb + j >= SR_KMAX) continue;
                int row, col;
                chunk_at(kb + j, row, col);
                nin[j]      = pl + (kb + j) * SR_PL < nch ? min(4, uw - 4 * col) : 0;
                const int y = ur.v_start + it.y0 + row, x = ur.h_start + 4 * col;
                xv[j]       = *(const uint2 *)(P.dxp + (size_t)y * P.fstride + x);
                advance();
            }
#pragma unroll
            for (int j = 0; j < LB2; j++) {
                const int kk = kb + j;
                if (kk >= SR_KMAX) break;
                // pixels outside the part read as zeros everywhere: g = 0 and (x - src) = 0 add nothing to any sum
                const uint32_t mlo = nin[j] >= 2 ? ~0u : nin[j] == 1 ? 0xFFFFu : 0u;
                const uint32_t mhi = nin[j] >= 4 ? ~0u : nin[j] == 3 ? 0xFFFFu : 0u;
                g[kk][0] &= mlo, g[kk][2] &= mlo, g[kk][1] &= mhi, g[kk][3] &= mhi;
                const uint2    x2 = make_uint2(xv[j].x & mlo, xv[j].y & mhi);
                const int      dxq[4] = {(int)(int16_t)(x2.x & 0xFFFF), (int)x2.x >> 16, (int)(int16_t)(x2.y & 0xFFFF),
                                         (int)x2.y >> 16};
                const uint32_t fw[4] = {__builtin_amdgcn_perm(g[kk][2], g[kk][0], 0x05040100u),
                                        __builtin_amdgcn_perm(g[kk][2], g[kk][0], 0x07060302u),
                                        __builtin_amdgcn_perm(g[kk][3], g[kk][1], 0x05040100u),
                                        __builtin_amdgcn_perm(g[kk][3], g[kk][1], 0x07060302u)};
                uint32_t m0 = 0, m1 = 0; // <= 4 g^2 < 2^32
                int      m3 = 0, m4 = 0; // |4 g s| < 2^31
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t gq = fw[q] & gmask; // (flt0 - u, flt1 - u); an ep's absent filter reads as 0
                    const int      g1 = (int)(int16_t)(gq & 0xFFFF), g2 = (int)gq >> 16, ss = -(dxq[q] << 4);
                    m0 += (uint32_t)(g1 * g1), m1 += (uint32_t)(g2 * g2);
                    m3 += g1 * ss, m4 += g2 * ss;
                    M2 += (unsigned long long)(long long)(g1 * g2);
                    g[kk][q] = gq;
                }
                M0 += m0, M1 += m1, M3 += (unsigned long long)(long long)m3, M4 += (unsigned long long)(long long)m4;
                sr_dx[kk * SR_PL + pl] = x2.x, sr_dx[(SR_KMAX + kk) * SR_PL + pl] = x2.y;
            }
        }
#endif
        {
            const unsigned long long t[5] = {wave_sum_u64_limbs(M0), wave_sum_u64_limbs(M1), wave_sum_u64_limbs(M2),
                                             wave_sum_u64_limbs(M3), wave_sum_u64_limbs(M4)};
            if ((pl & 63) == WAVE_LAST)
#pragma unroll
                for (int q = 0; q < 5; q++) s_red[pl >> 6][q] = t[q];
        }
        __syncthreads(); // B1: the moments are in s_red
        __syncthreads(); // B2: the first tree is in s_xq
        // diagnostics (stat): pixel wave 0's pass time (B2/B4 release to its arrival at B3) and its wait from B3 to the
        // B4 release
        unsigned long long tpass = 0, twait = 0, tmark = stat ? __builtin_amdgcn_s_memrealtime() : 0;
        if (!TREE && it.nparts == 1 && !(xmode & 0x200)) {
            // One barrier per pass, and no wave waits on another's descent step: every wave (pixel and control) holds
            // the seeded descent in its own scalar registers and steps it itself from the pass's wave partials --
            // report + next once per pass, the same decisions everywhere (the errors are the same LDS words).  Before
            // this the control wave stepped the descent and built both children of every candidate (three steps per
            // pass, serial) while the pixel waves waited at the barrier: 13 us of descent per item, 8 of them control
            Descent  Dw   = uniform(s_desc);
            bool     live = __builtin_amdgcn_readfirstlane(s_nv) != 0;
            uint32_t xq   = 0;
            {
                int32_t x[2];
                decode_xq(Dw, x);
                xq = __builtin_amdgcn_readfirstlane(pack2(x[0], x[1]));
            }
            for (int pass = 1; live; pass++) {
                const uint32_t xl[1] = {xq};
                sr_pass<1>(g, sr_dx, pl, K, 1, xl, s_red2[pass & 1]);
                if (stat) {
                    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                    tpass += t - tmark, tmark = t;
                }
                __syncthreads(); // B3: the pass's wave partials are in LDS
                unsigned long long e0 = 0;
#pragma unroll
                for (int w = 0; w < SR_PW; w++) e0 += s_red2[pass & 1][w][0];
                Dw.report(readlane64((long long)e0, 0));
                live = Dw.next() && pass <= SR_MAX_PASSES;
                if (live) {
                    int32_t x[2];
                    decode_xq(Dw, x);
                    xq = __builtin_amdgcn_readfirstlane(pack2(x[0], x[1]));
                }
                if (stat) {
                    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                    twait += t - tmark, tmark = t;
                }
            }
        } else if (!TREE && !(xmode & 0x200)) {
            // Row parts, self-stepping: the control wave sums this part's wave partials, exchanges the sum with the
            // other parts and leaves the frame-unit total in LDS (B4); then every wave steps its own copy of the
            // descent -- no children built, no wave waits on another's step
            Descent  Dw   = uniform(s_desc);
            bool     live = __builtin_amdgcn_readfirstlane(s_nv) != 0;
            uint32_t xq   = 0;
            {
                int32_t x[2];
                decode_xq(Dw, x);
                xq = __builtin_amdgcn_readfirstlane(pack2(x[0], x[1]));
            }
            for (int pass = 1; live; pass++) {
                const uint32_t xl[1] = {xq};
                sr_pass<1>(g, sr_dx, pl, K, 1, xl, s_red);
                if (stat) {
                    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                    tpass += t - tmark, tmark = t;
                }
                __syncthreads(); // B3: the pass's wave partials are in s_red
                __syncthreads(); // B4: the parts' total is in s_etot
                const bool okx = __builtin_amdgcn_readfirstlane(s_xok[pass & 1]) != 0;
                if (okx) {
                    Dw.report(readlane64((long long)s_etot[pass & 1], 0));
                    live = Dw.next() && pass <= SR_MAX_PASSES;
                } else
                    live = false;
                if (live) {
                    int32_t x[2];
                    decode_xq(Dw, x);
                    xq = __builtin_amdgcn_readfirstlane(pack2(x[0], x[1]));
                }
                if (stat) {
                    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                    twait += t - tmark, tmark = t;
                }
            }
        } else
        for (;;) {
            const int nv = __builtin_amdgcn_readfirstlane(s_nv);
            if (nv == 0) break;
            if constexpr (!TREE) {
                sr_pass<1>(g, sr_dx, pl, K, 1, s_xq, s_red);
            } else {
                switch (nv) {
                case 1: sr_pass<1>(g, sr_dx, pl, K, nv, s_xq, s_red); break;
                case 2: sr_pass<2>(g, sr_dx, pl, K, nv, s_xq, s_red); break;
                case 3: sr_pass<3>(g, sr_dx, pl, K, nv, s_xq, s_red); break;
                case 4: sr_pass<4>(g, sr_dx, pl, K, nv, s_xq, s_red); break;
                default: sr_pass<SG_NC>(g, sr_dx, pl, K, nv, s_xq, s_red); break;
                }
            }
            if (stat) {
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                tpass += t - tmark, tmark = t;
            }
            __syncthreads(); // B3: the pass's errors are in s_red
            __syncthreads(); // B4: the next tree (or the end) is in s_xq / s_nv
            if (stat) {
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                twait += t - tmark, tmark = t;
            }
        }
        if (stat && pl == 0) atomicAdd(stat + 7, tpass), atomicAdd(stat + 8, twait);
    } else {
        // ================= control wave =================
        // stat (SVTGPU_SR_STATS diagnostics, else null): items, passes, candidate-pixels, load / descent / control
        // ticks (100 MHz), pixels.  The control steps are the item's serial critical path: this wave issues ahead of
        // the other workgroup's pixel waves on its SIMD (it waits at the barriers otherwise)
        __builtin_amdgcn_s_setprio(3);
        const int                lane = threadIdx.x & 63;
        const unsigned long long t0   = stat ? __builtin_amdgcn_s_memrealtime() : 0;
        unsigned long long       tctl = 0, ncp = 0, tpre = 0;
        __syncthreads(); // B1
        const unsigned long long t1 = stat ? __builtin_amdgcn_s_memrealtime() : 0;
        long long v  = 0; // lane q < 5: moment q over the workgroup (and the other row parts)
        bool      ok = true;
        if (lane < 5) {
            unsigned long long t = 0;
            for (int w = 0; w < SR_PW; w++) t += s_red[w][lane];
            v = (long long)t;
            if (it.nparts > 1) ok = sr_exchange_lane(xch, it, 0, lane, v, status, xmode);
        }
        ok = __ballot(!ok) == 0;
        long long mv[5];
#pragma unroll
        for (int q = 0; q < 5; q++) mv[q] = readlane64(v, q);
        // the descent is wave-uniform from here on: kept in scalar registers, stepped by the scalar unit
        Descent D = uniform(sgr_seed(A, p, it.pair, (const int64_t *)mv, cfg));
        D.next(); // the seed itself is the first candidate
        sr_tree_publish(D, ok, nodes, s_xq, &s_mask, &s_nv);
        if (!TREE && it.nparts == 1 && !(xmode & 0x200)) {
            // the self-stepping path (see the pixel waves): the seeded descent to LDS for every wave, then the same
            // report + next per pass as everyone else
            if (lane == 0) s_desc = D;
            __syncthreads(); // B2
            bool live = ok;
            int  pass = 1;
            for (; live; pass++) {
                __syncthreads(); // B3
                const unsigned long long tb = stat ? __builtin_amdgcn_s_memrealtime() : 0;
                ncp += (unsigned long long)nch * 4;
                unsigned long long e0 = 0;
#pragma unroll
                for (int w = 0; w < SR_PW; w++) e0 += s_red2[pass & 1][w][0];
                D.report(readlane64((long long)e0, 0));
                live = D.next() && pass <= SR_MAX_PASSES;
                if (pass > SR_MAX_PASSES && lane == 0) atomicOr(status, 1);
                if (stat) tctl += __builtin_amdgcn_s_memrealtime() - tb;
            }
            if (stat && lane == 0) atomicAdd(stat + 1, (unsigned long long)(pass - 1));
        } else if (!TREE && nodes == 1 && !(xmode & 0x200)) {
            // self-stepping row parts (see the pixel waves): the exchange between B3 and B4, the step after B4
            if (lane == 0) s_desc = D;
            __syncthreads(); // B2
            bool live = ok;
            int  pass = 1;
            for (; live; pass++) {
                __syncthreads(); // B3
                const unsigned long long tb = stat ? __builtin_amdgcn_s_memrealtime() : 0;
                ncp += (unsigned long long)nch * 4;
                if (lane == 0) {
                    unsigned long long t = 0;
                    for (int w = 0; w < SR_PW; w++) t += s_red[w][0];
                    long long e   = (long long)t;
                    const bool ex = sr_exchange_lane(xch, it, pass, 0, e, status, xmode);
                    s_etot[pass & 1] = (unsigned long long)e, s_xok[pass & 1] = ex;
                }
                __syncthreads(); // B4
                const bool okx = __builtin_amdgcn_readfirstlane(s_xok[pass & 1]) != 0;
                if (okx) {
                    D.report(readlane64((long long)s_etot[pass & 1], 0));
                    live = D.next() && pass <= SR_MAX_PASSES;
                    if (pass > SR_MAX_PASSES && lane == 0) atomicOr(status, 1);
                } else
                    live = false;
                if (stat) tctl += __builtin_amdgcn_s_memrealtime() - tb;
            }
            if (stat && lane == 0) atomicAdd(stat + 1, (unsigned long long)(pass - 1));
        } else {
        __syncthreads(); // B2
        for (int pass = 1;; pass++) {
            const int nv = __builtin_amdgcn_readfirstlane(s_nv);
            if (nv == 0) break;
            const uint32_t mask = __builtin_amdgcn_readfirstlane(s_mask);
            uint32_t       xw = 0, xb = 0;
            bool           okw = false, okb = false;
            const unsigned long long tc0 = stat ? __builtin_amdgcn_s_memrealtime() : 0;
            if (nodes == 1) sr_children(D, xw, okw, xb, okb); // during the pass
            if (stat) tpre += __builtin_amdgcn_s_memrealtime() - tc0;
            __syncthreads(); // B3
            const unsigned long long tb = stat ? __builtin_amdgcn_s_memrealtime() : 0;
            ncp += (unsigned long long)nv * nch * 4;
            long long e = 0; // lane c < nv: compacted candidate c's error
            ok = true;
            if (lane < nv) {
                unsigned long long t = 0;
                for (int w = 0; w < SR_PW; w++) t += s_red[w][lane];
                e = (long long)t;
                if (it.nparts > 1) ok = sr_exchange_lane(xch, it, pass, lane, e, status, xmode);
            }
            ok = __ballot(!ok) == 0;
            if (pass > SR_MAX_PASSES) {
                if (lane == 0) atomicOr(status, 1);
                ok = false;
            }
            if (nodes == 1) { // the outcome picks a prepared child; the descent itself steps after the barrier
                const long long e0    = readlane64(e, 0);
                const bool      worse = !D.init && e0 > D.err;
                if (lane == 0) {
                    s_xq[0] = worse ? xw : xb;
                    s_mask  = 1;
                    s_nv    = ok && (worse ? okw : okb) ? 1 : 0;
                }
                if (stat) tctl += __builtin_amdgcn_s_memrealtime() - tb;
                __syncthreads(); // B4
                if (stat && lane == 0 && s_nv == 0) atomicAdd(stat + 1, (unsigned long long)pass);
                if (ok) { // the same state change as the choice above, with the error value kept
                    D.report(e0);
                    D.next();
                }
                continue;
            }
            if (ok) { // the same steps in every lane (the errors made uniform: scalar code)
                long long ev[SG_NC];
#pragma unroll
                for (int c = 0; c < SG_NC; c++) ev[c] = c < nv ? readlane64(e, c) : 0;
                sgr_replay(D, mask, [&](int node) {
                    const int i = __popc(mask & ((1u << node) - 1));
                    long long r = ev[0];
#pragma unroll
                    for (int c = 1; c < SG_NC; c++) r = i == c ? ev[c] : r;
                    return (int64_t)r;
                });
            }
            sr_tree_publish(D, ok && !D.done, nodes, s_xq, &s_mask, &s_nv);
            if (stat) tctl += __builtin_amdgcn_s_memrealtime() - tb;
            __syncthreads(); // B4
            if (stat && lane == 0 && s_nv == 0) atomicAdd(stat + 1, (unsigned long long)pass);
        }
        }
        if (lane == 0 && it.part == 0) ds[it.pair] = D;
        if (stat && lane == 0) {
            const unsigned long long te = __builtin_amdgcn_s_memrealtime();
            atomicAdd(stat + 0, 1ull), atomicAdd(stat + 2, ncp), atomicAdd(stat + 3, t1 - t0);
            atomicAdd(stat + 4, te - t1), atomicAdd(stat + 5, tctl);
            atomicAdd(stat + 6, (unsigned long long)nch * 4), atomicAdd(stat + 9, tpre);
            if (it.nparts > 1) // the row-part items apart: count, load, descent, control ticks
                atomicAdd(stat + 10, 1ull), atomicAdd(stat + 11, t1 - t0), atomicAdd(stat + 12, te - t1),
                    atomicAdd(stat + 13, tctl);
        }
    }
    PROF_END(tk);
}

struct Carver {
    size_t off = 0;
    size_t operator()(size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    }
};

// device-clock timing of the search's launches by kernel class (svtgpu_lr_profile).  Everything accumulates on the
// device: after a search one small kernel folds its launches' slots into per-class tick totals (and re-arms the
// slots), so a timed search adds no copies or host synchronization; the totals are read back only when asked for.
struct ProfClasses {
    uint8_t c[PROF_NL];
};
__global__ __launch_bounds__(PROF_NL) void prof_fold_kernel(unsigned long long *clk, int nl, const ProfClasses cls,
                                                            unsigned long long *acc) {
    const int i = threadIdx.x;
    if (i >= nl) return;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int k = 0; k < PROF_SP; k++) {
        t0 = min(t0, clk[i * PROF_SP + k]), t1 = max(t1, clk[(PROF_NL + i) * PROF_SP + k]);
        clk[i * PROF_SP + k] = ~0ull, clk[(PROF_NL + i) * PROF_SP + k] = 0;
    }
    if (t0 != ~0ull && t1 >= t0) atomicAdd(&acc[cls.c[i]], t1 - t0);
}

constexpr int NCLS = 6; // classes of SvtGpuLrProfile
struct LrProfiler {
    unsigned long long *d_clk = nullptr; // [PROF_NL][PROF_SP] workgroup starts (min), then the same of ends (max)
    unsigned long long *d_px  = nullptr; // [3][PROF_SP] evaluated pixels: trials, projection (pixel, ep), projection tiles
    unsigned long long *d_acc = nullptr; // [5] ticks per class, over the searches since the last read
    int                 nl = 0, searches = 0;
    ProfClasses         cls{};
    int32_t             launches[NCLS] = {0, 0, 0, 0, 0, 0};
    double              static_bytes[NCLS] = {0, 0, 0, 0, 0, 0}, bps = 2;
    bool                ok   = false;
    int32_t             mask = 63; // classes timed (bit c)
    bool                events = false; // bit 6 of the enable mask: HIP events around the timed launches too
    bool                serial = false; // bit 7: the Wiener chain on the caller's stream -- every kernel runs alone
    LrProfiler() {
        ok = hipMalloc(&d_clk, 16 * PROF_NL * PROF_SP) == hipSuccess && hipMalloc(&d_px, 24 * PROF_SP) == hipSuccess &&
             hipMalloc(&d_acc, 8 * NCLS) == hipSuccess && hipMemset(d_clk, 0xFF, 8 * PROF_NL * PROF_SP) == hipSuccess &&
             hipMemset(d_clk + PROF_NL * PROF_SP, 0, 8 * PROF_NL * PROF_SP) == hipSuccess &&
             hipMemset(d_px, 0, 24 * PROF_SP) == hipSuccess && hipMemset(d_acc, 0, 8 * NCLS) == hipSuccess &&
             hipDeviceSynchronize() == hipSuccess;
    }
    ~LrProfiler() {
        for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
        (void)hipFree(d_clk);
        (void)hipFree(d_px);
        (void)hipFree(d_acc);
    }
    // HIP events around every timed launch on its own stream: the launch duration as the command processor sees it
    // (rocprofv3's kernel trace measures the same span; the device clock above starts at the first workgroup and ends
    // at the last), summed per class at read time
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, int>> ev_used; // (class, index of the start event; the end event follows it)
    size_t                  ev_next = 0;
    int ev_begin(int c, hipStream_t st) {
        if (!events || !(mask >> c & 1)) return -1;
        while (ev_pool.size() < ev_next + 2) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return -1;
            ev_pool.push_back(e);
        }
        const int i = (int)ev_next;
        ev_next += 2;
        if (hipEventRecord(ev_pool[i], st) != hipSuccess) return -1;
        ev_used.push_back({c, i});
        return i;
    }
    void ev_end(int i, hipStream_t st) {
        if (i >= 0) (void)hipEventRecord(ev_pool[i + 1], st);
    }
    void start() { nl = 0; }
    // the timing slot of one launch of class c (nullptr: not timed)
    unsigned long long *slot(int c) {
        if (!(mask >> c & 1) || nl >= PROF_NL) return nullptr;
        cls.c[nl] = (uint8_t)c;
        launches[c]++;
        return d_clk + PROF_SP * nl++;
    }
    int finish(hipStream_t st) { // enqueued after the search's launches
        searches++;
        if (!nl) return SVTGPU_OK;
        hipLaunchKernelGGL(prof_fold_kernel, dim3(1), dim3(PROF_NL), 0, st, d_clk, nl, cls, d_acc);
        HIP_TRY(hipGetLastError());
        return SVTGPU_OK;
    }
    int read(SvtGpuLrProfile *out) { // totals since the last read, then reset
        unsigned long long acc[NCLS], pxs[3 * PROF_SP], px[3] = {0, 0, 0};
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(acc, d_acc, sizeof acc, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(pxs, d_px, sizeof pxs, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(d_acc, 0, sizeof acc));
        HIP_TRY(hipMemset(d_px, 0, sizeof pxs));
        HIP_TRY(hipDeviceSynchronize());
        for (int k = 0; k < 3 * PROF_SP; k++) px[k / PROF_SP] += pxs[k];
        std::memset(out, 0, sizeof *out);
        for (auto &u : ev_used) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, ev_pool[u.second], ev_pool[u.second + 1]) == hipSuccess) out->ms_events[u.first] += ms;
        }
        ev_used.clear(), ev_next = 0;
        for (int c = 0; c < NCLS; c++) {
            out->launches[c] = launches[c];
            out->ms[c]       = (float)(acc[c] * 1e-5); // 100 MHz ticks
            out->bytes[c]    = static_bytes[c];
        }
        out->bytes[2] += (double)px[0] * 2 * bps;                     // x and source per evaluated pixel
        out->bytes[3] += (double)px[1] * 4 + (double)px[2] * 2 * bps; // flt per (pixel, ep), x/source per tile
        out->searches = searches;
        searches      = 0;
        for (int c = 0; c < NCLS; c++) launches[c] = 0, static_bytes[c] = 0;
        return SVTGPU_OK;
    }
};

struct PlanePlan {
    int                  n = 0, nt = 0, unit_base = 0, tile_base = 0, win = 7, nval = 0, ne = 0, pair_base = 0;
    bool                 wn = false, sg = false;
    size_t               part_off = 0, mh_off = 0; // element offsets (int64)
    std::vector<int32_t> eps;
};

int plane_win(const SvtGpuLrSearchControls *c, int p) {
    const int win_l = c->wn_filter_tap_lvl == 1 ? 7 : c->wn_filter_tap_lvl == 2 ? 5 : 3;
    return p == 0 ? win_l : std::min(win_l, 5);
}

// RestUnitSearchInfo as rest_finish_search uses it (EbRestoration.h:349-360): best[] = best_rtype[WIENER - 1 ..
// SWITCHABLE - 1]
struct FinRusi {
    int64_t        sse[3];
    SvtGpuRestUnit wiener, sgrproj;
    int32_t        best[3];
};
// which finish passes of rest_finish_search run for plane p (force_restore_type_d and the per-plane skips,
// EbRestorationPick.c:1558-1560, 1597-1610): r 0 always; num_rtypes = 4 only with more than one unit
inline bool finish_runs(const SvtGpuLrSearchControls *c, int p, int n, int r) {
    const int force = c->wn_enabled ? (c->sg_enabled ? 4 : 1) : (c->sg_enabled ? 2 : 0);
    if (r == 3 && n <= 1) return false;
    if (force != 4 && r != 0 && r != force) return false;
    if (p && ((r == 1 && !c->wn_use_chroma) || (r == 2 && !c->sg_use_chroma))) return false;
    return true;
}

// rest_finish_search (EbRestorationPick.c:1555-1634) of plane p over its per-unit search records, on the host.  `rusi`
// is the reference's per-unit array, allocated once per frame (luma's unit count) and shared by the planes: each pass
// overwrites only what it computes, so a chroma plane's switchable pass reads luma's best_rtype / sse / wiener (or
// sgrproj) entries for a type that chroma does not search (search_switchable :1148-1200, copy_unit_info :1202-1209).
// Planes run in order 0, 1, 2 over the same array.
void finish_plane_shared(const SvtGpuLrSearchControls *c, int p, int win, const SvtGpuLrUnitSearch *rs, int n,
                         FinRusi *rusi, int32_t *frame_type, SvtGpuRestUnit *out) {
    double best_cost = 0;
    int    best_type = 0;
    for (int r = 0; r < 4; r++) {
        if (!finish_runs(c, p, n, r)) continue;
        SvtGpuRestUnit refw = default_wiener(), refs = default_sgrproj(); // rsc_on_tile
        int64_t        sse = 0, bits = 0;
        for (int u = 0; u < n; u++) {
            const SvtGpuLrUnitSearch &R = rs[u];
            FinRusi                  &Q = rusi[u];
            if (r == 0) { // search_norestore_finish
                Q.sse[0] = R.sse[0];
                sse += Q.sse[0];
            } else if (r == 1) { // search_wiener_finish
                const int64_t bn = c->wiener_restore_cost[0];
                Q.sse[1]         = R.sse[1];
                if (Q.sse[1] == INT64_MAX) {
                    bits += bn, sse += Q.sse[0], Q.best[0] = 0;
                    continue;
                }
                Q.wiener         = R.wiener;
                const int64_t bw = c->wiener_restore_cost[1] + ((int64_t)wiener_bits(win, Q.wiener, refw) << 9);
                const bool    t  = rdcost(c->rdmult, bw >> 4, Q.sse[1]) < rdcost(c->rdmult, bn >> 4, Q.sse[0]);
                Q.best[0]        = t ? 1 : 0;
                sse += Q.sse[t ? 1 : 0];
                bits += t ? bw : bn;
                if (t) refw = Q.wiener;
            } else if (r == 2) { // search_sgrproj_finish
                Q.sse[2] = R.sse[2], Q.sgrproj = R.sgrproj;
                const int64_t bn = c->sgrproj_restore_cost[0];
                const int64_t bs = c->sgrproj_restore_cost[1] + ((int64_t)sgrproj_bits(Q.sgrproj, refs) << 9);
                const bool    t  = rdcost(c->rdmult, bs >> 4, Q.sse[2]) < rdcost(c->rdmult, bn >> 4, Q.sse[0]);
                Q.best[1]        = t ? 2 : 0;
                sse += Q.sse[t ? 2 : 0];
                bits += t ? bs : bn;
                if (t) refs = Q.sgrproj;
            } else { // search_switchable (7 / 5 Wiener taps by plane)
                double  bc = 0;
                int64_t bb = 0;
                int     bt = 0;
                for (int t = 0; t < 3; t++) {
                    if (t > 0 && Q.best[t - 1] == 0) continue;
                    const int64_t cp = t == 1 ? wiener_bits(p == 0 ? 7 : 5, Q.wiener, refw) : t == 2 ? sgrproj_bits(Q.sgrproj, refs) : 0;
                    const int64_t b  = c->switchable_restore_cost[t] + (cp << 9);
                    const double  cost = rdcost(c->rdmult, b >> 4, Q.sse[t]);
                    if (t == 0 || cost < bc) bc = cost, bb = b, bt = t;
                }
                Q.best[2] = bt;
                sse += Q.sse[bt];
                bits += bb;
                if (bt == 1) refw = Q.wiener;
                if (bt == 2) refs = Q.sgrproj;
            }
        }
        const double cost = rdcost(c->rdmult, bits >> 4, sse);
        if (r == 0 || cost < best_cost) best_cost = cost, best_type = r;
    }
    *frame_type = best_type;
    for (int u = 0; u < n; u++) { // copy_unit_info
        std::memset(&out[u], 0, sizeof out[u]);
        if (best_type) {
            const int t = rusi[u].best[best_type - 1];
            out[u]      = t == 1 ? rusi[u].wiener : rusi[u].sgrproj;
            out[u].type = t;
        }
    }
}

// the whole frame's finish on the host: planes [0, nplanes) in order over one shared array
void finish_frame_host(const SvtGpuLrSearchControls *c, int nplanes, const int32_t *n, const SvtGpuLrUnitSearch *const *rs,
                       int32_t *frame_type, SvtGpuRestUnit *const *out) {
    std::vector<FinRusi> rusi((size_t)std::max(1, n[0]));
    std::memset(rusi.data(), 0, sizeof(FinRusi) * rusi.size());
    for (int p = 0; p < nplanes; p++)
        finish_plane_shared(c, p, plane_win(c, p), rs[p], n[p], rusi.data(), &frame_type[p], out[p]);
}

// ---------------------------------------------------------------------------------------------
// rest_finish_search on the device (round 6; the host form above stays behind SVTGPU_LR_FINISH=host).
// The reference's finish is sequential over a plane's units because every unit's Wiener / self-guided rate is coded
// against the last unit that took that filter (rsc->wiener / rsc->sgrproj).  A lane stepping that chain with the
// rate arithmetic inside would be slower than the host; instead
//   lr_records_kernel      the per-unit records (SvtGpuLrUnitSearch) from the search's device results -- what the host
//                          read-back assembled -- into one array of all planes' units (the gather a tiled picture
//                          all-reduces);
//   lr_fin_tables_kernel   one wave per unit evaluates, for every reference the chain can hold at that unit (the 63
//                          units before it and the default), the pass's decision: search_wiener_finish /
//                          search_sgrproj_finish as bits of a 64-bit mask; for search_switchable the costs of the
//                          Wiener and the self-guided choice against each of those references (the choice needs one
//                          of each: two tables of 64 doubles instead of a 64 x 64 table);
//   lr_fin_walk_kernel     one workgroup walks the chains -- per unit a mask bit (two table entries and two compares)
//                          selected by how far back the reference is, the tables staged in LDS a chunk of units at a
//                          time -- evaluating a decision directly only when the reference lies outside the tabulated
//                          window; then the per-unit rates of the taken path
//                          in parallel, each pass's frame cost, the frame types and copy_unit_info into the state's
//                          units.  The decisions are the reference's own comparisons (RDCOST_DBL in double,
//                          -ffp-contract=off), so the walk takes exactly the reference's path.
// The shared RestUnitSearchInfo array (finish_plane_shared) is modelled by reading luma's entries for a type a chroma
// plane does not search.
// ---------------------------------------------------------------------------------------------
constexpr int FIN_K1 = 63; // r = 1 / 2 masks: bit k < 63 = the unit k + 1 back as the reference, bit 63 = the default
constexpr int FIN_CH = 64; // the walks: units per chunk (a lane per unit; the switchable tables staged in LDS)
constexpr int FIN_OUT = 8; // device result words: frame types [3], search status, sequence

struct RecArgs {
    int32_t                   nplanes, n_all, wn[3], sg[3];
    const unsigned long long *sse0, *sse2;
    const SvtGpuRestUnit     *wu;
    const Descent            *wds;
    const int32_t            *best, *raw;
    const int32_t            *dst; // record index of every searched unit
    SvtGpuLrUnitSearch       *rec;
};
__global__ __launch_bounds__(256) void lr_records_kernel(const SearchArgs A, const RecArgs R) {
    const int gu = blockIdx.x * 256 + threadIdx.x;
    if (gu >= R.n_all) return;
    int p = 0;
    while (p + 1 < R.nplanes && gu >= A.pl[p + 1].unit_base) p++;
    SvtGpuLrUnitSearch o;
    memset(&o, 0, sizeof o);
    o.sse[0] = (int64_t)R.sse0[gu];
    o.sse[1] = INT64_MAX;
    if (R.wn[p] && R.wu[gu].type) {
        const Descent &d = R.wds[gu];
        o.sse[1]         = d.err;
        o.wiener         = R.wu[gu];
        int v[3];
        d.taps(0, v), set_wiener_taps(o.wiener.hfilter, v);
        d.taps(1, v), set_wiener_taps(o.wiener.vfilter, v);
    }
    if (R.sg[p]) { // sgr_best_kernel: the first ep of least error and its descent's two values
        o.sgrproj.type   = SVTGPU_RESTORE_SGRPROJ;
        o.sgrproj.ep     = A.pl[p].eps[R.best[4 * gu]];
        o.sgrproj.xqd[0] = R.raw[2 * gu], o.sgrproj.xqd[1] = R.raw[2 * gu + 1];
        o.sse[2]         = (int64_t)R.sse2[gu];
    }
    R.rec[R.dst[gu]] = o;
}

struct FinPlane {
    int32_t n, base;   // units of the plane; its first record (and table entry)
    int32_t run[4];    // the finish passes that run (finish_runs)
    int32_t win1;      // search_wiener_finish's window (plane_win); search_switchable uses 7 luma / 5 chroma
    int32_t own1, own2; // the shared rusi's Wiener / self-guided entries are this plane's own (else luma's)
};
struct FinArgs {
    FinPlane                  pl[3];
    int32_t                   nplanes, nrec, rdmult, sw[3], wn[2], sg[2];
    const SvtGpuLrUnitSearch *rec;
    unsigned long long       *m1, *m2;
    uint8_t                  *b1, *b2; // switchable: the Wiener / self-guided coefficient bits [unit][64] (< 2^8)
    int32_t                  *path;   // [4][nrec]: r 1, r 2, r 3 (Wiener ref), r 3 (self-guided ref): choice | (ref + 1) << 2
    SvtGpuRestUnit           *units;  // the state's units (d_units[0]: the planes back to back, the records' layout)
    int32_t                  *out;    // [FIN_OUT] device results
    int32_t                  *out_host; // mapped pinned copy
    const int32_t            *wstat, *sstat; // the descents' status words (wiener_res / sgr_res) or null
    int32_t                   seq;
    unsigned long long       *clk; // diagnostics (SVTGPU_LR_FIN_CLK): the walk's phase ends on s_memrealtime, or null
    int32_t                   wtab; // the walks read the tables for references up to wtab units back (FIN_K1; tests:
                                    // SVTGPU_LR_FIN_WIN = 1 sends nearly every step to the evaluation at the step)
};

// the shared rusi entries of unit u of plane p a switchable pass and copy_unit_info read
__device__ inline const SvtGpuLrUnitSearch &fin_rec(const FinArgs &F, int p, int u) { return F.rec[F.pl[p].base + u]; }
__device__ inline const SvtGpuLrUnitSearch &fin_w(const FinArgs &F, int p, int u) { return fin_rec(F, F.pl[p].own1 ? p : 0, u); }
__device__ inline const SvtGpuLrUnitSearch &fin_s(const FinArgs &F, int p, int u) { return fin_rec(F, F.pl[p].own2 ? p : 0, u); }

// search_wiener_finish's decision at unit u with the reference unit `ref` (-1: the default)
__device__ bool fin_accept1(const FinArgs &F, int p, int u, int ref) {
    const SvtGpuLrUnitSearch &R = fin_rec(F, p, u);
    if (R.sse[1] == INT64_MAX) return false;
    const SvtGpuRestUnit rw = ref < 0 ? default_wiener() : fin_rec(F, p, ref).wiener;
    const int64_t        bw = F.wn[1] + ((int64_t)wiener_bits(F.pl[p].win1, R.wiener, rw) << 9);
    return rdcost(F.rdmult, bw >> 4, R.sse[1]) < rdcost(F.rdmult, (int64_t)F.wn[0] >> 4, R.sse[0]);
}
// search_sgrproj_finish's decision
__device__ bool fin_accept2(const FinArgs &F, int p, int u, int ref) {
    const SvtGpuLrUnitSearch &R = fin_rec(F, p, u);
    const SvtGpuRestUnit      rs = ref < 0 ? default_sgrproj() : fin_rec(F, p, ref).sgrproj;
    const int64_t             bs = F.sg[1] + ((int64_t)sgrproj_bits(R.sgrproj, rs) << 9);
    return rdcost(F.rdmult, bs >> 4, R.sse[2]) < rdcost(F.rdmult, (int64_t)F.sg[0] >> 4, R.sse[0]);
}
// search_switchable's costs of types 1 and 2 against the references rw / rs
__device__ double fin_c1(const FinArgs &F, int p, int u, int rw) {
    const SvtGpuRestUnit r = rw < 0 ? default_wiener() : fin_w(F, p, rw).wiener;
    const int64_t        b = F.sw[1] + ((int64_t)wiener_bits(p == 0 ? 7 : 5, fin_w(F, p, u).wiener, r) << 9);
    return rdcost(F.rdmult, b >> 4, fin_w(F, p, u).sse[1]);
}
__device__ double fin_c2(const FinArgs &F, int p, int u, int rs) {
    const SvtGpuRestUnit r = rs < 0 ? default_sgrproj() : fin_s(F, p, rs).sgrproj;
    const int64_t        b = F.sw[2] + ((int64_t)sgrproj_bits(fin_s(F, p, u).sgrproj, r) << 9);
    return rdcost(F.rdmult, b >> 4, fin_s(F, p, u).sse[2]);
}
__device__ inline double fin_c0(const FinArgs &F, int p, int u) {
    return rdcost(F.rdmult, (int64_t)F.sw[0] >> 4, fin_rec(F, p, u).sse[0]);
}
// the rate term of RDCOST_DBL for the bits sw + (coef << 9) (rdcost's first addend, the same operations)
__device__ inline double fin_rate(int rdmult, int sw, int coef) {
    const int64_t b = sw + ((int64_t)coef << 9);
    return ((double)(b >> 4) * rdmult) / (double)(1 << 9);
}
// the choice (t == 0 || cost < best, in type order) with types 1 / 2 allowed by a1 / a2
__device__ inline int fin_pick(double c0, double c1, double c2, bool a1, bool a2) {
    int    bt = 0;
    double bc = c0;
    if (a1 && c1 < bc) bt = 1, bc = c1;
    if (a2 && c2 < bc) bt = 2;
    return bt;
}

__global__ __launch_bounds__(64) void lr_fin_tables_kernel(const FinArgs F) {
    const int b = blockIdx.x, lane = threadIdx.x;
    int       p = 0;
    while (p + 1 < F.nplanes && b >= F.pl[p + 1].base) p++;
    const FinPlane &P = F.pl[p];
    const int       u = b - P.base;
    if (u >= P.n) return;
    const int ref = lane < FIN_K1 ? u - 1 - lane : -1; // lane k: the unit k + 1 back; lane 63: the default
    const bool ok = lane == FIN_K1 || ref >= 0;
    for (int r = 1; r <= 2; r++) {
        if (!P.run[r]) continue;
        const bool a = ok && (r == 1 ? fin_accept1(F, p, u, ref) : fin_accept2(F, p, u, ref));
        const unsigned long long m = __ballot(a);
        if (lane == 0) (r == 1 ? F.m1 : F.m2)[b] = m;
    }
    if (!P.run[3]) return;
    // the switchable pass's coefficient bits against each candidate reference (its costs are formed in the walk)
    int c1 = 0, c2 = 0;
    if (ok) {
        const SvtGpuRestUnit rw = ref < 0 ? default_wiener() : fin_w(F, p, ref).wiener;
        const SvtGpuRestUnit rs = ref < 0 ? default_sgrproj() : fin_s(F, p, ref).sgrproj;
        c1 = wiener_bits(p == 0 ? 7 : 5, fin_w(F, p, u).wiener, rw);
        c2 = sgrproj_bits(fin_s(F, p, u).sgrproj, rs);
    }
    F.b1[(size_t)b * 64 + lane] = (uint8_t)c1;
    F.b2[(size_t)b * 64 + lane] = (uint8_t)c2;
}

// a wave-uniform 64-bit value held by lane i of v
__device__ inline unsigned long long lane_u64(unsigned long long v, int i) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, i);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), i);
    return ((unsigned long long)hi << 32) | lo;
}

// a wave-uniform double held by lane i of v
__device__ inline double lane_f64(double v, int i) { return __builtin_bit_cast(double, lane_u64(__builtin_bit_cast(unsigned long long, v), i)); }

// The chains are walked by one wave each, a chunk of FIN_CH units at a time, a lane per unit of the chunk.  A unit's
// decision against its reference comes from the tables when the reference is one of the 63 units before it or the
// default (a bit of the unit's mask, or its coefficient bits in LDS); a reference further back can only be the one the
// chain held when the chunk began (a reference taken inside the chunk is at most 62 units back), so every unit of the
// chunk is evaluated against that one at the chunk's start, lane-parallel.  A step reads no global memory and waits
// on no evaluation (only the test window SVTGPU_LR_FIN_WIN < 63 reaches the evaluation at the step).

// the r = 1 / r = 2 chain of plane p: path[u] = decision | (reference + 1) << 2
__device__ void fin_walk12(const FinArgs &F, int p, int r, int lane) {
    const FinPlane           &P    = F.pl[p];
    const unsigned long long *M    = (r == 1 ? F.m1 : F.m2) + P.base;
    int32_t                  *path = F.path + (size_t)(r - 1) * F.nrec + P.base;
    int                       ref  = -1;
    for (int u0 = 0; u0 < P.n; u0 += FIN_CH) {
        const int                nl = min(FIN_CH, P.n - u0);
        const unsigned long long mv = lane < nl ? M[u0 + lane] : 0ull;
        const int                ref0 = ref; // the chunk's units against the chain's reference at its start
        const bool sa = ref0 >= 0 && lane < nl && (r == 1 ? fin_accept1(F, p, u0 + lane, ref0) : fin_accept2(F, p, u0 + lane, ref0));
        const unsigned long long spec = __ballot(sa);
        int                      pv = 0;
        for (int i = 0; i < nl; i++) {
            const int u = u0 + i, k = ref < 0 ? FIN_K1 : u - 1 - ref;
            bool      a;
            if (ref < 0 || k < F.wtab) a = (lane_u64(mv, i) >> k) & 1; // bit FIN_K1: the default
            else if (ref == ref0) a = (spec >> i) & 1;
            else a = r == 1 ? fin_accept1(F, p, u, ref) : fin_accept2(F, p, u, ref);
            // uniform (every lane takes the same decision): a scalar, so the chain's branches are scalar branches
            a = __builtin_amdgcn_readfirstlane((int)a) != 0;
            if (lane == i) pv = (int)a | ((ref + 1) << 2);
            if (a) ref = u;
        }
        if (lane < nl) path[u0 + lane] = pv;
    }
}

// the switchable chain of plane p: path[2][u] / path[3][u] = choice | (Wiener / self-guided ref + 1) << 2.  lb1 / lb2:
// the wave's LDS for the chunk's coefficient bits [FIN_CH][64]
__device__ void fin_walk3(const FinArgs &F, int p, int lane, uint8_t *lb1, uint8_t *lb2, const double *rate1,
                          const double *rate2) {
    const FinPlane &P  = F.pl[p];
    const int32_t  *d1 = F.path + F.pl[P.own1 ? p : 0].base, *d2 = F.path + F.nrec + F.pl[P.own2 ? p : 0].base;
    int32_t        *pw = F.path + 2 * (size_t)F.nrec + P.base, *ps = F.path + 3 * (size_t)F.nrec + P.base;
    int             rw = -1, rs = -1;
    for (int u0 = 0; u0 < P.n; u0 += FIN_CH) {
        const int nl = min(FIN_CH, P.n - u0);
        const unsigned long long tc0 = F.clk && p == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
        // the chunk's bit rows (64 B per unit and table), 16-B pieces; then per lane its unit's cost terms
        for (int q = lane; q < nl * 4; q += 64) {
            const size_t row = (size_t)(P.base + u0 + (q >> 2)) * 64;
            ((uint4 *)lb1)[q] = ((const uint4 *)(F.b1 + row))[q & 3];
            ((uint4 *)lb2)[q] = ((const uint4 *)(F.b2 + row))[q & 3];
        }
        const int rw0 = rw, rs0 = rs; // the chunk's units against the chain's references at its start (far ones)
        double    c0v = 0, s1v = 0, s2v = 0, f1v = 0, f2v = 0;
        int       a1v = 0, a2v = 0;
        if (lane < nl) {
            const int u = u0 + lane;
            c0v = fin_c0(F, p, u);
            s1v = (double)fin_w(F, p, u).sse[1] * (1 << 7); // rdcost's second addend
            s2v = (double)fin_s(F, p, u).sse[2] * (1 << 7);
            a1v = d1[u] & 1, a2v = d2[u] & 1;
            if (rw0 >= 0) f1v = fin_c1(F, p, u, rw0);
            if (rs0 >= 0) f2v = fin_c2(F, p, u, rs0);
        }
        __builtin_amdgcn_wave_barrier(); // the wave's LDS stores before its loads (in order within a wave)
        unsigned long long tc1 = 0;
        if (F.clk && p == 0) { // diagnostics: luma's chunk preparation / step loop
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            tc1 = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) F.clk[5] += tc1 - tc0, F.clk[7] += 1;
        }
        int qw = 0, qs = 0;
        for (int i = 0; i < nl; i++) {
            const int  u  = u0 + i;
            const bool a1 = __builtin_amdgcn_readlane(a1v, i) != 0, a2 = __builtin_amdgcn_readlane(a2v, i) != 0;
            const int  kw = rw < 0 ? FIN_K1 : u - 1 - rw, ks = rs < 0 ? FIN_K1 : u - 1 - rs;
            // the rate terms of all 256 coefficient-bit counts are tabulated (rate1 / rate2): two dependent LDS reads
            const double c1 = rw < 0 || kw < F.wtab ? rate1[lb1[i * 64 + kw]] + lane_f64(s1v, i)
                            : rw == rw0             ? lane_f64(f1v, i)
                                                    : fin_c1(F, p, u, rw);
            const double c2 = rs < 0 || ks < F.wtab ? rate2[lb2[i * 64 + ks]] + lane_f64(s2v, i)
                            : rs == rs0             ? lane_f64(f2v, i)
                                                    : fin_c2(F, p, u, rs);
            // uniform: a scalar (otherwise the chain's references live in VGPRs and every branch on them is exec-masked)
            const int    bt = __builtin_amdgcn_readfirstlane(fin_pick(lane_f64(c0v, i), c1, c2, a1, a2));
            if (lane == i) qw = bt | ((rw + 1) << 2), qs = bt | ((rs + 1) << 2);
            if (bt == 1) rw = u;
            if (bt == 2) rs = u;
        }
        if (F.clk && p == 0 && lane == 0) F.clk[6] += __builtin_amdgcn_s_memrealtime() - tc1;
        if (lane < nl) pw[u0 + lane] = qw, ps[u0 + lane] = qs;
        __builtin_amdgcn_wave_barrier(); // this chunk's LDS reads before the next chunk's stores
    }
}

constexpr int FIN_NT = 1024; // the walk kernel's lanes: six / three walking waves, then all of them for the sums
__global__ __launch_bounds__(FIN_NT) void lr_fin_walk_kernel(const FinArgs F) {
    __shared__ unsigned long long acc[3][4][2]; // per plane and pass: sse, bits
    __shared__ int32_t            ft[3];
    __shared__ __attribute__((aligned(16))) uint8_t lb[3][2][FIN_CH * 64]; // fin_walk3's staging, per wave
    __shared__ double rate[2][256]; // fin_rate of the switchable Wiener / self-guided costs for every bit count < 2^8
    // the wave index through readfirstlane: the compiler then knows each walk's plane, unit count and loop bounds are
    // wave-uniform, and keeps the chains' references in SGPRs with scalar branches (from threadIdx.x >> 6 it treated
    // the loops as divergent and every step as exec-masked vector code)
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (tid < 24) (&acc[0][0][0])[tid] = 0;
    if (F.clk && tid == 0) F.clk[0] = __builtin_amdgcn_s_memrealtime(), F.clk[5] = F.clk[6] = F.clk[7] = 0;
    if (tid < 512) rate[tid >> 8][tid & 255] = fin_rate(F.rdmult, F.sw[1 + (tid >> 8)], tid & 255); // read after the barrier
    // the r = 1 / 2 chains (wave 2 p + r - 1: independent of each other), then the switchable chains (which read the
    // r = 1 / 2 outcomes, luma's for a type chroma does not search)
    if (wv < 2 * F.nplanes && F.pl[wv >> 1].run[1 + (wv & 1)]) fin_walk12(F, wv >> 1, 1 + (wv & 1), lane);
    __syncthreads();
    if (F.clk && tid == 0) F.clk[1] = __builtin_amdgcn_s_memrealtime();
    if (wv < F.nplanes && F.pl[wv].run[3]) fin_walk3(F, wv, lane, lb[wv][0], lb[wv][1], rate[0], rate[1]);
    __syncthreads();
    if (F.clk && tid == 0) F.clk[2] = __builtin_amdgcn_s_memrealtime();
    // the rate and distortion of every unit on each pass's path, summed per (plane, pass): one pass over the items of
    // all planes (item i: plane p, pass r, unit u)
    const int n0 = 4 * F.pl[0].n, n1 = n0 + 4 * F.pl[1].n, nall = F.nplanes > 2 ? n1 + 4 * F.pl[2].n : F.nplanes > 1 ? n1 : n0;
    for (int i = tid; i < nall; i += FIN_NT) {
        const int p = i < n0 ? 0 : i < n1 ? 1 : 2, j = i - (p == 0 ? 0 : p == 1 ? n0 : n1);
        const FinPlane &P = F.pl[p];
        const int r = j / P.n, u = j - r * P.n;
        if (!P.run[r]) continue;
        const SvtGpuLrUnitSearch &R = fin_rec(F, p, u);
        int64_t                   sse = 0, bits = 0;
        if (r == 0) {
            sse = R.sse[0];
        } else if (r <= 2) {
            const int32_t q = F.path[(size_t)(r - 1) * F.nrec + P.base + u];
            const int     ref = (q >> 2) - 1;
            if (!(q & 1)) {
                sse = R.sse[0], bits = r == 1 ? F.wn[0] : F.sg[0];
            } else if (r == 1) {
                const SvtGpuRestUnit rw = ref < 0 ? default_wiener() : fin_rec(F, p, ref).wiener;
                sse = R.sse[1], bits = F.wn[1] + ((int64_t)wiener_bits(P.win1, R.wiener, rw) << 9);
            } else {
                const SvtGpuRestUnit rs = ref < 0 ? default_sgrproj() : fin_rec(F, p, ref).sgrproj;
                sse = R.sse[2], bits = F.sg[1] + ((int64_t)sgrproj_bits(R.sgrproj, rs) << 9);
            }
        } else {
            const int32_t qw = F.path[2 * (size_t)F.nrec + P.base + u], qs = F.path[3 * (size_t)F.nrec + P.base + u];
            const int     bt = qw & 3, rw = (qw >> 2) - 1, rs = (qs >> 2) - 1;
            int64_t       cp = 0;
            if (bt == 1) {
                const SvtGpuRestUnit r0 = rw < 0 ? default_wiener() : fin_w(F, p, rw).wiener;
                cp = wiener_bits(p == 0 ? 7 : 5, fin_w(F, p, u).wiener, r0), sse = fin_w(F, p, u).sse[1];
            } else if (bt == 2) {
                const SvtGpuRestUnit r0 = rs < 0 ? default_sgrproj() : fin_s(F, p, rs).sgrproj;
                cp = sgrproj_bits(fin_s(F, p, u).sgrproj, r0), sse = fin_s(F, p, u).sse[2];
            } else {
                sse = R.sse[0];
            }
            bits = F.sw[bt] + (cp << 9);
        }
        atomicAdd(&acc[p][r][0], (unsigned long long)sse);
        atomicAdd(&acc[p][r][1], (unsigned long long)bits);
    }
    __syncthreads();
    if (F.clk && tid == 0) F.clk[3] = __builtin_amdgcn_s_memrealtime();
    if (tid < 3) { // each pass's frame cost; the first of least cost (r == 0 || cost < best)
        int best = 0;
        if (tid < F.nplanes) {
            double bc = 0;
            for (int r = 0; r < 4; r++) {
                if (!F.pl[tid].run[r]) continue;
                const double c = rdcost(F.rdmult, (int64_t)acc[tid][r][1] >> 4, (int64_t)acc[tid][r][0]);
                if (r == 0 || c < bc) bc = c, best = r;
            }
        }
        ft[tid] = best;
    }
    __syncthreads();
    if (F.clk && tid == 0) F.clk[4] = __builtin_amdgcn_s_memrealtime();
    // copy_unit_info into the state's units (every plane; zero where the frame type is NONE): one pass over all units
    const int m0 = F.pl[0].n, m1 = m0 + F.pl[1].n, mall = m1 + F.pl[2].n;
    for (int i = tid; i < mall; i += FIN_NT) {
        const int       p = i < m0 ? 0 : i < m1 ? 1 : 2, u = i - (p == 0 ? 0 : p == 1 ? m0 : m1);
        const FinPlane &P = F.pl[p];
        SvtGpuRestUnit  o;
        memset(&o, 0, sizeof o);
        if (p < F.nplanes && ft[p]) {
            const int32_t q = F.path[(size_t)(ft[p] - 1) * F.nrec + P.base + u];
            const int     t = ft[p] == 3 ? (q & 3) : (q & 1) ? ft[p] : 0;
            o               = t == 1 ? fin_w(F, p, u).wiener : fin_s(F, p, u).sgrproj;
            o.type          = t;
        }
        F.units[P.base + u] = o;
    }
    if (tid < FIN_OUT) {
        const int32_t v = tid < 3   ? ft[tid]
                        : tid == 3 ? (F.wstat && *F.wstat ? 1 : 0) | (F.sstat && *F.sstat ? 2 : 0)
                        : tid == 4 ? F.seq
                                   : 0;
        F.out[tid] = v;
        if (F.out_host) __hip_atomic_store(&F.out_host[tid], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <typename Fn>
void launch_stats(int win, Fn &&f) {
    if (win == 7) f(std::integral_constant<int, 7>());
    else if (win == 5) f(std::integral_constant<int, 5>());
    else f(std::integral_constant<int, 3>());
}

// largest Wiener window staged in LDS (SVTGPU_WR_LDS_CAP overrides: measurements of the global-memory path)
int wr_lds_cap() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_WR_LDS_CAP");
        return e ? std::atoi(e) : WR_LDS_CAP;
    }();
    return v;
}

// largest row part of the resident self-guided search (pixels); SVTGPU_SR_PART_PX lowers it (tests of the parted path)
int sr_part_px() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_SR_PART_PX");
        return e ? std::max(64, std::min(std::atoi(e), SR_MAX_PX)) : SR_MAX_PX;
    }();
    return v;
}

// candidates per pass of the resident self-guided search: a complete speculative tree of 1, 3 or 7 nodes
// (SVTGPU_SR_TREE for A/B measurements).  One: the descent's own candidate sequence, 7.1 passes per (unit, ep) at 4K
// against 3.9 (3 nodes) and 2.7 (7 nodes) -- the resident passes are cheap, and a larger tree's evaluated-but-unused
// candidates cost the other frames' work at three frames in flight (2366 / 2321 Mpx/s for 1 / 3 nodes,
// profiles/r03/srvar)
int sr_tree_nodes() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_SR_TREE");
        const int   n = e ? std::atoi(e) : 1;
        return n == 3 || n == 7 ? n : 1;
    }();
    return v;
}

// The statistics of one unit on the matrix cores (svt_av1_compute_stats(_highbd) for 8- and 10-bit samples: the
// RTCD shim of lr_shims.hip): the unit, its source and a 3-sample border are staged as a small frame (the border
// replicated past the reference's `half` samples, which no feature of a smaller window reads), cut into <= 64 x 64
// tiles, run through wiener_stats_kernel and summed per entry; M and H are assembled exactly as wiener_solve_kernel
// does, each int64 total divided once (EbRestorationPick.c:671-760).
template <typename T>
int stats_unit_mfma(int win, const T *dgd, const T *src, int h_start, int h_end, int v_start, int v_end,
                    int dgd_stride, int src_stride, int64_t *M, int64_t *H, int div) {
    static_assert(sizeof(T) <= 2, "8- or 16-bit samples");
    const int half = win >> 1, w = h_end - h_start, h = v_end - v_start;
    if (w <= 0 || h <= 0 || (win != 7 && win != 5 && win != 3)) return SVTGPU_ERR_INVALID_ARG;
    const int FW = ((w + 3) & ~3) + 3 + 8, FH = h + 6; // staged frame: unit at (3, 3); 4-aligned source rows + slack
    std::vector<T> fd((size_t)FW * FH), fs((size_t)FW * FH, (T)0);
    unsigned long long sum = 0;
    for (int y = -3; y < h + 3; y++) {
        const int yy = std::min(std::max(y, -half), h - 1 + half); // the rows the reference may read
        const T  *row = dgd + (long)(v_start + yy) * dgd_stride + h_start;
        for (int x = -3; x < FW - 3; x++) fd[(size_t)(y + 3) * FW + x + 3] = row[std::min(std::max(x, -half), w - 1 + half)];
    }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            fs[(size_t)(y + 3) * FW + x + 3] = src[(long)(v_start + y) * src_stride + h_start + x];
            sum += dgd[(long)(v_start + y) * dgd_stride + h_start + x];
        }
    std::vector<Tile> tiles;
    for (int y = 0; y < h; y += 64)
        for (int x = 0; x < w; x += 64) tiles.push_back({0, 0, 3 + x, 3 + y, std::min(64, w - x), std::min(64, h - y)});
    const URect u{3, 3 + w, 3, 3 + h};
    const int   nt = (int)tiles.size(), npair = win * (win + 1) / 2, nval = (npair + 1) * 49;
    Carver      c;
    const size_t o_d = c(sizeof(T) * fd.size()), o_s = c(sizeof(T) * fs.size()), o_t = c(sizeof(Tile) * nt),
                 o_u = c(sizeof(URect)), o_t0 = c(8), o_sum = c(8), o_part = c(8 * (size_t)nt * nval);
    static thread_local void  *buf = nullptr;
    static thread_local size_t cap = 0;
    if (c.off > cap) {
        if (buf) (void)hipFree(buf);
        buf = nullptr, cap = 0;
        HIP_TRY(hipMalloc(&buf, c.off));
        cap = c.off;
    }
    uint8_t    *d  = (uint8_t *)buf;
    hipStream_t st = svtgpu_shim_stream();
    const int32_t t0[2] = {0, nt};
    HIP_TRY(hipMemcpyAsync(d + o_d, fd.data(), sizeof(T) * fd.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d + o_s, fs.data(), sizeof(T) * fs.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d + o_t, tiles.data(), sizeof(Tile) * nt, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d + o_u, &u, sizeof u, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d + o_t0, t0, 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d + o_sum, &sum, 8, hipMemcpyHostToDevice, st));
    SearchArgs A;
    std::memset(&A, 0, sizeof A);
    PlaneArgs &P = A.pl[0];
    P.dgd = d + o_d, P.src = d + o_s, P.dstride = P.sstride = FW, P.W = FW, P.H = FH;
    P.bd = sizeof(T) == 1 ? 8 : 10, P.win = win, P.nval = nval;
    A.tiles = (const Tile *)(d + o_t), A.units = (const URect *)(d + o_u), A.tile0 = (const int32_t *)(d + o_t0);
    launch_stats(win, [&](auto wc) {
        hipLaunchKernelGGL((wiener_stats_kernel<T, decltype(wc)::value>), dim3(nt), dim3(256), 0, st, A, 0,
                           (const unsigned long long *)(d + o_sum), (long long *)(d + o_part), nullptr);
    });
    HIP_TRY(hipGetLastError());
    std::vector<long long> part((size_t)nt * nval);
    HIP_TRY(hipMemcpyAsync(part.data(), d + o_part, 8 * part.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<long long> blk(nval, 0);
    for (int t = 0; t < nt; t++)
        for (int k = 0; k < nval; k++) blk[k] += part[(size_t)t * nval + k];
    const int win2 = win * win;
    for (int k = 0; k < win2; k++) M[k] = blk[npair * 49 + (k / win) * 7 + k % win] / div;
    for (int t = 0; t < win2 * win2; t++) { // H[k][l]: k = ck * win + rk (the reference's y[] order)
        const int k = t / win2, l = t % win2, ck = k / win, rk = k % win, cl = l / win, rl = l % win;
        const int c1 = std::min(ck, cl), c2 = std::max(ck, cl), r1 = ck <= cl ? rk : rl, r2 = ck <= cl ? rl : rk;
        H[t] = blk[(c1 * win - c1 * (c1 - 1) / 2 + (c2 - c1)) * 49 + r1 * 7 + r2] / div;
    }
    return SVTGPU_OK;
}

// plane p's Wiener window for the controls

// The search of the units in unit rows [rb[p], re[p]) of planes 0..nplanes-1.  frame_type != nullptr: the band
// is the whole frame and the RD finish runs and sets the state's units.
// waits for the last device finish queued on `st` (bounded when an exchange sits before it) and returns its frame
// types, or the failure a resident descent reported (status words copied by lr_fin_walk_kernel)
int lr_collect(SvtGpuLrState *s, hipStream_t st, int32_t *frame_type) {
    if (int rc = svtgpu_comm_wait(s->comm, st)) return rc;
    s->fin_pending            = 0;
    const volatile int32_t *o = s->h_fout;
    if (o[4] != s->fin_seq) {
        svtgpu_set_last_hip_error(hipErrorUnknown, "LR device finish: result word missing after the stream wait",
                                  __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    if (o[3]) {
        svtgpu_set_last_hip_error(hipErrorUnknown, (o[3] & 1) ? "LR Wiener descent: round bound or part exchange timed out"
                                                              : "LR self-guided descent: pass bound, part plan or exchange failed",
                                  __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    for (int p = 0; p < 3; p++) s->last_ft[p] = o[p];
    if (frame_type)
        for (int p = 0; p < 3; p++) frame_type[p] = o[p];
    return SVTGPU_OK;
}

// SVTGPU_LR_FINISH=host: rest_finish_search on the host after a read-back of the records (the round-5 form; A/B)
bool lr_finish_on_host() {
    static const bool h = [] {
        const char *e = std::getenv("SVTGPU_LR_FINISH");
        return e && !std::strcmp(e, "host");
    }();
    return h;
}

// fin == 0: the records come back to the host (search_out) and, for the whole frame (frame_type != nullptr), the RD
// finish runs there.  fin == 1: the records and the RD finish stay on the device (a tiled picture all-reduces the
// records on the device first), the state's units are written in stream order; frame_type != nullptr then waits for
// the result and reads the frame types (and the records into search_out), nullptr returns at once (the asynchronous
// search: svtgpu_lr_read_result collects it).
template <typename T>
int search_frame(SvtGpuLrState *s, const SvtGpuFrame *rec, const SvtGpuFrame *src, const SvtGpuLrSearchControls *c,
                 int nplanes, const int32_t *rb, const int32_t *re, const int32_t *cb, const int32_t *ce,
                 int32_t *frame_type, SvtGpuLrUnitSearch *const *search_out, hipStream_t st, int fin = 0) {
    // SVTGPU_LR_TIMING=1 prints the host-side phase times (wall clock, including the waits) to stderr
    static const bool timing = std::getenv("SVTGPU_LR_TIMING") != nullptr;
    auto              clk    = [] { return std::chrono::steady_clock::now(); };
    auto              t_last = clk();
    double            t_ph[6] = {0, 0, 0, 0, 0, 0};
    auto              mark   = [&](int i) {
        const auto now = clk();
        t_ph[i] += std::chrono::duration<double, std::milli>(now - t_last).count();
        t_last = now;
    };
    // ---- plan: units (foreach_rest_unit_in_tile, EbRestoration.c:1257-1294), their <= 64x64 tiles, the eps ----
    PlanePlan            pp[3];
    std::vector<URect>   units;
    std::vector<Tile>    tiles;
    std::vector<int32_t> tile0, uloc; // uloc: plane-local index of every global unit
    int                  npairs = 0, n_wn = 0, nt_wn = 0, n_sg = 0, nt_sg = 0, sg_planes = 0;
    size_t               flt_elems = 0, part_elems = 0, mh_elems = 0;
    for (int p = 0; p < nplanes; p++) {
        PlanePlan &q = pp[p];
        const int  W = lr_plane_w(s, p), H = lr_plane_h(s, p), usz = s->unit_size[p], ext = usz * 3 / 2, off = 8 >> (p > 0);
        q.unit_base = (int)units.size(), q.tile_base = (int)tiles.size();
        int urow = 0, uidx = 0;
        for (int y0 = 0; y0 < H; urow++) {
            const int uh = (H - y0 < ext) ? H - y0 : usz;
            int       vs = std::max(0, y0 - off), ve = y0 + uh;
            if (ve < H) ve -= off;
            for (int x0 = 0, ucol = 0; x0 < W; uidx++, ucol++) {
                const int uw = (W - x0 < ext) ? W - x0 : usz;
                if (urow >= rb[p] && urow < re[p] && ucol >= cb[p] && ucol < ce[p]) {
                    tile0.push_back((int)tiles.size());
                    for (int y = vs; y < ve; y += 64)
                        for (int x = x0; x < x0 + uw; x += 64)
                            tiles.push_back({p, (int)units.size(), x, y, std::min(64, x0 + uw - x), std::min(64, ve - y)});
                    units.push_back({x0, x0 + uw, vs, ve});
                    uloc.push_back(uidx);
                }
                x0 += uw;
            }
            y0 += uh;
        }
        q.n = (int)units.size() - q.unit_base, q.nt = (int)tiles.size() - q.tile_base;
        if (urow != s->vunits[p] || uidx != s->hunits[p] * s->vunits[p]) return SVTGPU_ERR_INVALID_ARG;
        q.wn   = c->wn_enabled && (!p || c->wn_use_chroma);
        q.win  = plane_win(c, p);
        q.nval = (q.win * (q.win + 1) / 2 + 1) * 49;
        if (c->sg_enabled && (!p || c->sg_use_chroma))
            for (int e = c->sg_start_ep[p > 0]; e < c->sg_end_ep[p > 0]; e += std::max(1, c->sg_ep_inc[p > 0]))
                q.eps.push_back(e);
        q.ne = (int)q.eps.size(), q.sg = q.ne > 0;
        q.pair_base = npairs;
        npairs += q.n * q.ne;
        if (q.wn) {
            n_wn += q.n, nt_wn += q.nt;
            q.part_off = part_elems, q.mh_off = mh_elems;
            part_elems += (size_t)q.nt * q.nval, mh_elems += (size_t)q.n * q.nval;
        }
        if (q.sg) {
            n_sg += q.n, nt_sg += q.nt, sg_planes++;
            flt_elems += (size_t)(q.ne * 2 + 1) * ((W + 63) & ~63) * H; // the eps' g planes and the dx plane
        }
    }
    tile0.push_back((int)tiles.size());
    for (const Tile &t : tiles) // 4-pixel chunks start on tile x offsets (unit columns: multiples of 32)
        if (t.x0 & 3) return SVTGPU_ERR_UNSUPPORTED;
    const int n_all = (int)units.size(), nt_all = (int)tiles.size();
    if (n_all == 0) return SVTGPU_OK; // an empty band
    // the records' layout: every plane's units back to back (the state's units, d_units[0]); dst[gu]: the record of
    // searched unit gu
    int32_t nrec = 0, rbase[3];
    for (int p = 0; p < 3; p++) rbase[p] = nrec, nrec += s->hunits[p] * s->vunits[p];
    std::vector<int32_t> dst(n_all);
    for (int p = 0, gu = 0; p < nplanes; p++)
        for (int u = 0; u < pp[p].n; u++, gu++) dst[gu] = rbase[p] + uloc[gu];
    // the resident Wiener kernel takes every unit whose rows fit its registers (all units of the 4K / 1080p frames);
    // its workgroups start with the largest units (the longest chains); windows up to WR_LDS_CAP live in LDS
    // The resident Wiener kernel takes every unit up to 384 columns wide (unit sizes <= 256): a unit is cut into the
    // fewest row parts that fit one CU's LDS and registers each (global-memory mode when no cut up to WR_MAX_PARTS
    // does); workgroups start with the largest parts (the longest chains), the parts of a unit adjacent.
    std::vector<WrItem> wr_items;
    bool                wr_parted = false;
    int                 wr_lds = 0;
    {
        std::vector<int> ord(n_wn);
        std::vector<int> np(n_wn, 1);
        for (int u = 0; u < n_wn; u++) {
            const URect &r = units[u];
            const int    w = r.h_end - r.h_start, h = r.v_end - r.v_start;
            ord[u]         = u;
            int k = 1;
            while (k < WR_MAX_PARTS && !wr_lds_mode(w, (h + k - 1) / k, wr_lds_cap())) k++;
            np[u] = wr_lds_mode(w, (h + k - 1) / k, wr_lds_cap()) ? k : 1;
            if (np[u] > 1) wr_parted = true;
            const int hp = (h + np[u] - 1) / np[u];
            if (wr_lds_mode(w, hp, wr_lds_cap())) wr_lds = std::max(wr_lds, wr_window_bytes(w, hp));
        }
        auto part_area = [&](int u) {
            return (units[u].h_end - units[u].h_start) * ((units[u].v_end - units[u].v_start + np[u] - 1) / np[u]);
        };
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return part_area(a) > part_area(b); });
        for (int u : ord) {
            const int h = units[u].v_end - units[u].v_start, first = (int)wr_items.size();
            for (int k = 0; k < np[u]; k++)
                wr_items.push_back({u, h * k / np[u], h * (k + 1) / np[u], k, np[u], first});
        }
    }
    const int n_wr = (int)wr_items.size();
    // The resident self-guided search (sgr_res_kernel): one item per (unit row part, ep).  Workgroups are dealt
    // round-robin over the 8 XCDs (block b on XCD b mod 8), so the grid is laid out as 8 lanes (positions r, r + 8, ...):
    // a unit's items -- its eps, and the row parts of each -- go to one lane, consecutively.  The eps of a unit then
    // read its CDEF and source samples through one L2, and the parts of an item sit next to each other in their XCD's
    // in-order dispatch, so a waiting part's partners are always dispatched after it (never behind other waiting
    // parts).  Units are dealt largest first to the lane with the least work; empty slots (pair -1) pad the lanes.
    std::vector<SrItem>  sr_items;
    bool                 sr_parted = false;
    if (npairs) {
        std::vector<std::vector<SrItem>> lanes(8);
        std::vector<long long>           load(8, 0);
        std::vector<int>                 ord;
        for (int p = 0; p < nplanes; p++)
            if (pp[p].sg)
                for (int u = 0; u < pp[p].n; u++) ord.push_back(pp[p].unit_base + u);
        auto area = [&](int u) { return (long long)(units[u].h_end - units[u].h_start) * (units[u].v_end - units[u].v_start); };
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return area(a) > area(b); });
        for (int u : ord) {
            int p = 0;
            while (p + 1 < nplanes && u >= pp[p + 1].unit_base) p++;
            const PlanePlan &q = pp[p];
            const int        cw = (units[u].h_end - units[u].h_start + 3) >> 2, h = units[u].v_end - units[u].v_start;
            const int        maxrows = std::max(1, sr_part_px() / 4 / std::max(cw, 1)), np = (h + maxrows - 1) / maxrows;
            if (np > SR_MAX_PARTS) return SVTGPU_ERR_UNSUPPORTED; // a unit wider than 1024 x 4 samples per row part
            sr_parted |= np > 1;
            const int lane = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            for (int k = 0; k < q.ne; k++) {
                const int first = (int)lanes[lane].size(); // lane-local; made global below
                for (int part = 0; part < np; part++)
                    lanes[lane].push_back({q.pair_base + (u - q.unit_base) * q.ne + k, h * part / np, h * (part + 1) / np,
                                           part, np, first});
            }
            load[lane] += area(u) * q.ne;
        }
        size_t len = 0;
        for (auto &l : lanes) len = std::max(len, l.size());
        sr_items.assign(8 * len, SrItem{-1, 0, 0, 0, 1, 0});
        for (int r = 0; r < 8; r++)
            for (size_t m = 0; m < lanes[r].size(); m++) {
                SrItem it = lanes[r][m];
                it.first  = 8 * it.first + r; // parts of an item: positions first, first + 8, ...
                sr_items[8 * m + r] = it;
            }
    }
    const int n_sr = (int)sr_items.size();
    // ---- device scratch and pinned staging ----
    // three contiguous spans keep the host traffic to one copy each: the plan (uploaded when it changes), the
    // accumulators zeroed per search, the results read back (o_sse is the last zeroed and the first read)
    Carver       dc;
    const size_t o_tiles = dc(sizeof(Tile) * nt_all), o_units = dc(sizeof(URect) * n_all), o_t0 = dc(4 * (n_all + 1)),
                 o_witem = dc(sizeof(WrItem) * (size_t)n_wr), o_sritem = dc(sizeof(SrItem) * (size_t)n_sr),
                 o_dst = dc(4 * (size_t)n_all);
    const size_t plan_span = dc.off;
    // zeroed per search: the accumulators, the device finish's records (zero-padded: a tiled picture sums them) and
    // paths (a pass that does not run reads as "none taken")
    const size_t o_sum = dc(8 * n_all), o_rec = dc(sizeof(SvtGpuLrUnitSearch) * (size_t)nrec),
                 o_path = dc(16 * (size_t)nrec), o_sse = dc(8 * n_all), o_sse2 = dc(8 * (size_t)n_sg), o_wstat = dc(8),
                 o_sstat = dc(8);
    const size_t zero_span = dc.off - o_sum;
    const size_t o_wu = dc(sizeof(SvtGpuRestUnit) * n_wn), o_wds = dc(sizeof(Descent) * n_wn),
                 o_best = dc(16 * (size_t)n_sg), o_braw = dc(8 * (size_t)n_sg);
    const size_t res_span = dc.off - o_sse; // the (unit, ep) descents stay on the device: the best ep's come back
    const size_t o_sds = dc(sizeof(Descent) * npairs);
    const size_t o_part = dc(8 * part_elems), o_mh = dc(8 * mh_elems);
    const size_t o_m1 = dc(8 * (size_t)nrec), o_m2 = dc(8 * (size_t)nrec), o_b1 = dc(64 * (size_t)nrec),
                 o_b2 = dc(64 * (size_t)nrec), o_fout = dc(4 * FIN_OUT);
    // the uncached arena: the SSE exchange words of the Wiener units cut into row parts (wiener_res_kernel)
    Carver       qc;
    const size_t q_wrx = qc(16 * (size_t)n_wr), q_srx = qc(128 * (size_t)n_sr);
    Carver       hc; // host mirrors of the plan and result spans keep the device layout
    const size_t h_plan = hc(plan_span), h_res = hc(res_span), h_cnt = hc(32), h_out = hc(sizeof(SvtGpuRestUnit) * n_all),
                 h_rec = hc(sizeof(SvtGpuLrUnitSearch) * (size_t)nrec);
    const size_t h_sse = h_res, h_sse2 = h_res + (o_sse2 - o_sse), h_wu = h_res + (o_wu - o_sse),
                 h_wds = h_res + (o_wds - o_sse), h_best = h_res + (o_best - o_sse), h_braw = h_res + (o_braw - o_sse);
    if (dc.off > s->work_bytes) {
        (void)hipFree(s->d_work);
        s->d_work = nullptr, s->work_bytes = 0;
        HIP_TRY(hipMalloc(&s->d_work, dc.off));
        s->work_bytes = dc.off;
        s->plan_bytes.clear(); // nothing uploaded into the new buffer yet
    }
    if (s->pin_free) HIP_TRY(hipEventSynchronize(s->pin_free)); // the previous search's upload has read h_pin
    if (hc.off > s->pin_bytes) {
        if (s->h_pin) (void)hipHostFree(s->h_pin);
        s->h_pin = nullptr, s->pin_bytes = 0;
        HIP_TRY(hipHostMalloc(&s->h_pin, hc.off, hipHostMallocDefault));
        s->pin_bytes = hc.off;
    }
    if (2 * flt_elems > s->flt_bytes) {
        (void)hipFree(s->d_flt);
        s->d_flt = nullptr, s->flt_bytes = 0;
        HIP_TRY(hipMalloc(&s->d_flt, 2 * flt_elems));
        s->flt_bytes = 2 * flt_elems;
    }
    uint8_t *wb = (uint8_t *)s->d_work, *hb = (uint8_t *)s->h_pin;
    auto     dp = [&](size_t o) { return (void *)(wb + o); };
    auto     hp = [&](size_t o) { return (void *)(hb + o); };
    SearchArgs A;
    std::memset(&A, 0, sizeof A);
    size_t flt_off = 0;
    for (int p = 0; p < nplanes; p++) {
        PlaneArgs &P = A.pl[p];
        P.dgd = rec->plane[p], P.src = src->plane[p], P.dstride = rec->stride[p], P.sstride = src->stride[p];
        P.W = lr_plane_w(s, p), P.H = lr_plane_h(s, p), P.bd = rec->bit_depth, P.fstride = (P.W + 63) & ~63;
        P.flt       = s->d_flt + flt_off;
        P.unit_base = pp[p].unit_base, P.pair_base = pp[p].pair_base, P.ne = pp[p].ne;
        for (int k = 0; k < pp[p].ne; k++) {
            P.eps[k] = pp[p].eps[k], P.f1e[k] = k;
            for (int j = 0; j < k; j++)
                if (kHostSgrR[P.eps[k]][1] && kHostSgrS1[P.eps[j]] == kHostSgrS1[P.eps[k]]) {
                    P.f1e[k] = j;
                    break;
                }
        }
        P.win = pp[p].win, P.nval = pp[p].nval, P.mh_off = (int64_t)pp[p].mh_off;
        P.dxp = pp[p].sg ? P.flt + (size_t)pp[p].ne * 2 * P.fstride * P.H : nullptr;
        if (pp[p].sg) flt_off += (size_t)(pp[p].ne * 2 + 1) * P.fstride * P.H;
    }
    A.tiles = (const Tile *)dp(o_tiles), A.units = (const URect *)dp(o_units), A.tile0 = (const int32_t *)dp(o_t0);
    auto *d_t0 = (int32_t *)dp(o_t0);
    // ---- phase 1: sums, Wiener statistics, self-guided filters and moments ----
    LrProfiler         *prof = (LrProfiler *)s->prof;
    unsigned long long *pc   = prof ? prof->d_px : nullptr;
    auto run = [&](int c, hipStream_t ls, auto &&launch) {
        const int ev = prof ? prof->ev_begin(c, ls) : -1;
        launch(prof ? prof->slot(c) : nullptr);
        if (prof) prof->ev_end(ev, ls);
    };
    if (prof) prof->start();
    {
        uint8_t *pl = (uint8_t *)hp(h_plan);
        std::memset(pl, 0, plan_span);
        std::memcpy(pl + o_tiles, tiles.data(), sizeof(Tile) * nt_all);
        std::memcpy(pl + o_units, units.data(), sizeof(URect) * n_all);
        std::memcpy(pl + o_t0, tile0.data(), 4 * (n_all + 1));
        std::memcpy(pl + o_witem, wr_items.data(), sizeof(WrItem) * (size_t)n_wr);
        std::memcpy(pl + o_sritem, sr_items.data(), sizeof(SrItem) * (size_t)n_sr);
        std::memcpy(pl + o_dst, dst.data(), 4 * (size_t)n_all);
        if (s->plan_work != s->d_work || s->plan_bytes.size() != plan_span ||
            std::memcmp(s->plan_bytes.data(), pl, plan_span)) { // a new plan: one upload
            HIP_TRY(hipMemcpyAsync(dp(0), pl, plan_span, hipMemcpyHostToDevice, st));
            svtgpu_count_xfer(0, plan_span);
            s->plan_bytes.assign(pl, pl + plan_span);
            s->plan_work = s->d_work;
        }
    }
    // Every accumulator, status word and exchange arena is zeroed here, before the first kernel: a memset queued
    // behind the filters would wait for a CU slot while the resident Wiener descent holds them (~140 us at 4K).
    HIP_TRY(hipMemsetAsync(dp(o_sum), 0, zero_span, st));
    uint8_t *qa = nullptr;
    if ((n_wn && wr_parted) || (n_sr && sr_parted)) {
        if (qc.off > s->qarena_bytes) {
            if (s->d_qarena) (void)hipFree(s->d_qarena);
            s->d_qarena = nullptr, s->qarena_bytes = 0;
            HIP_TRY(hipExtMallocWithFlags(&s->d_qarena, qc.off, hipDeviceMallocUncached));
            s->qarena_bytes = qc.off;
        }
        qa = (uint8_t *)s->d_qarena;
        HIP_TRY(hipMemsetAsync(qa, 0, qc.off, st));
    }
    // the self-guided row parts' exchange words: uncached memory (default) or, with SVTGPU_SR_XCH=l2, cached memory that
    // stays in the XCD's L2 (no memset: the search epoch tags the words)
    static const bool sr_l2 = [] {
        const char *e = std::getenv("SVTGPU_SR_XCH");
        return e && !std::strcmp(e, "l2");
    }();
    unsigned sr_xmode = 0;
    if (n_sr && sr_parted && sr_l2) {
        const size_t need = 128 * (size_t)n_sr;
        if (need > s->sxarena_bytes) {
            if (s->d_sxarena) (void)hipFree(s->d_sxarena);
            s->d_sxarena = nullptr, s->sxarena_bytes = 0;
            HIP_TRY(hipMalloc(&s->d_sxarena, need));
            HIP_TRY(hipMemsetAsync(s->d_sxarena, 0, need, st));
            s->sxarena_bytes = need;
        }
        // the tag holds 8 epoch bits: when they wrap, clear the arena so no word left 256 searches ago passes for this
        // one's.  Test-only mode: the words are visible to an item's parts only through one XCD's L2, which
        // holds while workgroups are dealt round-robin over the 8 XCDs (SPX partition mode, positions first + 8 q);
        // another placement makes the partner polls time out (status word -> SVTGPU_ERR_HIP), never a wrong sum
        if ((++s->sx_epoch & 0xFFu) == 0) {
            HIP_TRY(hipMemsetAsync(s->d_sxarena, 0, s->sxarena_bytes, st));
            ++s->sx_epoch;
        }
        sr_xmode = 0x100u | (s->sx_epoch & 0xFFu);
    }
    static const bool sr_two_barriers = [] { // SVTGPU_SR_1B=0 (A/B): every item on the two-barrier path, the control
        const char *e = std::getenv("SVTGPU_SR_1B"); // wave stepping the descent alone (round 3's form)
        return e && !std::strcmp(e, "0");
    }();
    if (sr_two_barriers) sr_xmode |= 0x200u;
    static const bool wr_classic = [] { // SVTGPU_WR_CLASSIC=1 (A/B): the round-4 Wiener step (thread 0, two barriers)
        const char *e = std::getenv("SVTGPU_WR_CLASSIC");
        return e && std::atoi(e) != 0;
    }();
    static const bool   wr_stats = std::getenv("SVTGPU_WR_STATS") != nullptr; // per-search diagnostics to stderr
    static unsigned long long *wr_stat = nullptr;
    if (wr_stats && !wr_stat) HIP_TRY(hipMalloc(&wr_stat, 128));
    if (wr_stat) HIP_TRY(hipMemsetAsync(wr_stat, 0, 128, st));
    static const bool   sr_stats = std::getenv("SVTGPU_SR_STATS") != nullptr; // per-search diagnostics to stderr
    static unsigned long long *sr_stat = nullptr;
    if (sr_stats && !sr_stat) HIP_TRY(hipMalloc(&sr_stat, 128));
    if (sr_stat) HIP_TRY(hipMemsetAsync(sr_stat, 0, 128, st));
    run(0, st, [&](unsigned long long *tk) {
        hipLaunchKernelGGL(unit_sums_kernel<T>, dim3(nt_all), dim3(256), 0, st, A, (unsigned long long *)dp(o_sum),
                           (unsigned long long *)dp(o_sse), tk);
    });
    HIP_TRY(hipGetLastError());
    // The Wiener chain (statistics, decomposition, trial rounds) and the self-guided chain (filters, seeds,
    // projection rounds) are independent until the RD finish: the Wiener chain runs on a second stream, so its
    // latency-bound rounds fill the gaps of the self-guided work and the other way round.
    // measurement (svtgpu_lr_profile bit 7): both chains on the caller's stream, so a kernel's duration is its own,
    // not its share of the CUs beside the other chain's kernels
    const bool serial = prof && prof->serial;
    if (!s->wst && !serial)
        if (int rc = lr_make_wiener_stream(s)) return rc;
    hipStream_t sw     = serial ? st : s->wst;
    if (!serial) {
        HIP_TRY(hipEventRecord(s->ev_fork, st));
        HIP_TRY(hipStreamWaitEvent(sw, s->ev_fork, 0));
    }
    for (int p = 0; p < nplanes; p++) {
        const PlanePlan &q = pp[p];
        if (!q.wn) continue;
        long long *part = (long long *)dp(o_part) + q.part_off, *mh = (long long *)dp(o_mh) + q.mh_off;
        run(0, sw, [&](unsigned long long *tk) {
            launch_stats(q.win, [&](auto wc) {
                hipLaunchKernelGGL((wiener_stats_kernel<T, decltype(wc)::value>), dim3(q.nt), dim3(256), 0, sw, A,
                                   q.tile_base, (const unsigned long long *)dp(o_sum), part, tk);
            });
        });
        run(0, sw, [&](unsigned long long *tk) {
            hipLaunchKernelGGL(reduce_parts_kernel, dim3(q.n, (q.nval + 255) / 256), dim3(256), 0, sw, (const long long *)part,
                               (const int32_t *)d_t0 + q.unit_base, q.tile_base, q.nval, mh, tk);
        });
        HIP_TRY(hipGetLastError());
    }
    if (nt_sg) {
        run(1, st, [&](unsigned long long *tk) { hipLaunchKernelGGL(sgr_flt_kernel<T>, dim3(nt_sg), dim3(SG_NT), 0, st, A, tk); });
        HIP_TRY(hipGetLastError());
    }
    mark(0);
    // ---- phase 2: descent seeds (Wiener decomposition per unit, projection solve per (unit, ep)) ----
    SeedCfg cfg;
    cfg.wn_use_refinement = c->wn_use_refinement, cfg.wn_max_one_step = c->wn_max_one_refinement_step;
    cfg.sg_refine[0] = c->sg_refine[0], cfg.sg_refine[1] = c->sg_refine[1];
    if (n_wn) {
        run(4, sw, [&](unsigned long long *tk) {
            hipLaunchKernelGGL(wiener_solve_kernel, dim3(n_wn), dim3(256), 0, sw, A, nplanes, (const int64_t *)dp(o_mh),
                               cfg, (Descent *)dp(o_wds), (SvtGpuRestUnit *)dp(o_wu), tk);
        });
        HIP_TRY(hipGetLastError());
    }
    mark(1);
    // ---- phase 3: descent rounds on the device ----
    if (n_wn) { // the whole Wiener descent of every unit, resident on one CU each (or a few, for the largest)
        run(2, sw, [&](unsigned long long *tk) {
            hipLaunchKernelGGL(wiener_res_kernel<T>, dim3(n_wr), dim3(WR_NT), wr_lds, sw, A, (Descent *)dp(o_wds),
                               (const WrItem *)dp(o_witem), wr_lds, (unsigned long long *)(qa ? qa + q_wrx : nullptr),
                               (int32_t *)dp(o_wstat), pc, wr_stat, tk, (int)wr_classic);
        });
        HIP_TRY(hipGetLastError());
    }
    if (n_sr) { // the whole self-guided search of every (unit, ep), resident on one CU each (or a few)
        run(3, st, [&](unsigned long long *tk) {
            const int nodes = sr_tree_nodes();
            auto kern = nodes == 1 ? sgr_res_kernel<T, false> : sgr_res_kernel<T, true>;
            hipLaunchKernelGGL(kern, dim3(n_sr), dim3(SR_NT), SR_LDS, st, A, sg_planes,
                               (const SrItem *)dp(o_sritem), cfg, nodes, (Descent *)dp(o_sds),
                               (unsigned long long *)(sr_parted ? (sr_l2 ? (uint8_t *)s->d_sxarena : qa + q_srx) : nullptr),
                               sr_xmode, (int32_t *)dp(o_sstat), sr_stat, tk);
        });
        HIP_TRY(hipGetLastError());
    }
    mark(2);
    // ---- phase 4: best ep and its clipped SSE; read back the descents ----
    if (n_sg) {
        hipLaunchKernelGGL(sgr_best_kernel, dim3((n_sg + 255) / 256), dim3(256), 0, st, (const Descent *)dp(o_sds), A,
                           sg_planes, n_sg, (int32_t *)dp(o_best), (int32_t *)dp(o_braw));
        run(4, st, [&](unsigned long long *tk) {
            hipLaunchKernelGGL(sgr_sse_kernel<T>, dim3(nt_sg), dim3(256), 0, st, A, (const int32_t *)dp(o_best),
                               (unsigned long long *)dp(o_sse2), tk);
        });
        HIP_TRY(hipGetLastError());
    }
    if (!serial) {
        HIP_TRY(hipEventRecord(s->ev_join, sw)); // the Wiener chain joins the caller's stream
        HIP_TRY(hipStreamWaitEvent(st, s->ev_join, 0));
    }
    if (prof)
        if (int rc = prof->finish(st)) return rc; // fold the launch timings on the device, no read-back
    if (fin) { // ---- phase 5 on the device: the records, [the gather,] rest_finish_search ----
        if (!s->h_fout) {
            HIP_TRY(hipHostMalloc((void **)&s->h_fout, 4 * FIN_OUT, hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(s->h_fout, 0, 4 * FIN_OUT);
            HIP_TRY(hipHostGetDevicePointer((void **)&s->h_fout_dev, s->h_fout, 0));
        }
        RecArgs R;
        std::memset(&R, 0, sizeof R);
        R.nplanes = nplanes, R.n_all = n_all;
        for (int p = 0; p < nplanes; p++) R.wn[p] = pp[p].wn, R.sg[p] = pp[p].sg;
        R.sse0 = (const unsigned long long *)dp(o_sse), R.sse2 = (const unsigned long long *)dp(o_sse2);
        R.wu = (const SvtGpuRestUnit *)dp(o_wu), R.wds = (const Descent *)dp(o_wds);
        R.best = (const int32_t *)dp(o_best), R.raw = (const int32_t *)dp(o_braw);
        R.dst = (const int32_t *)dp(o_dst), R.rec = (SvtGpuLrUnitSearch *)dp(o_rec);
        hipLaunchKernelGGL(lr_records_kernel, dim3((n_all + 255) / 256), dim3(256), 0, st, A, R);
        HIP_TRY(hipGetLastError());
        // a picture tiled over GPUs: the zero-padded records summed over the ranks = the gather rest_finish_search reads
        // (one contributor per unit), on the device: no host wait
        static_assert(sizeof(SvtGpuLrUnitSearch) % 8 == 0, "records travel as uint64 words");
        if (svtgpu_comm_tiled(s->comm))
            if (int rc = svtgpu_comm_sum(s->comm, dp(o_rec), (size_t)nrec * sizeof(SvtGpuLrUnitSearch) / 8, true, st,
                                         SVTGPU_XCH_LR))
                return rc;
        FinArgs F;
        std::memset(&F, 0, sizeof F);
        bool tables = false;
        for (int p = 0; p < 3; p++) {
            FinPlane &P = F.pl[p];
            P.n = s->hunits[p] * s->vunits[p], P.base = rbase[p];
            for (int r = 0; r < 4; r++) P.run[r] = p < nplanes && finish_runs(c, p, P.n, r);
            P.win1 = plane_win(c, p);
            P.own1 = p == 0 || P.run[1], P.own2 = p == 0 || P.run[2];
            tables |= P.run[1] || P.run[2] || P.run[3];
        }
        F.nplanes = nplanes, F.nrec = nrec, F.rdmult = c->rdmult;
        for (int k = 0; k < 3; k++) F.sw[k] = c->switchable_restore_cost[k];
        for (int k = 0; k < 2; k++) F.wn[k] = c->wiener_restore_cost[k], F.sg[k] = c->sgrproj_restore_cost[k];
        F.rec = (const SvtGpuLrUnitSearch *)dp(o_rec);
        F.m1 = (unsigned long long *)dp(o_m1), F.m2 = (unsigned long long *)dp(o_m2);
        F.b1 = (uint8_t *)dp(o_b1), F.b2 = (uint8_t *)dp(o_b2);
        F.path = (int32_t *)dp(o_path), F.units = s->d_units[0];
        F.out = (int32_t *)dp(o_fout), F.out_host = s->h_fout_dev;
        F.wstat = n_wn ? (const int32_t *)dp(o_wstat) : nullptr, F.sstat = n_sr ? (const int32_t *)dp(o_sstat) : nullptr;
        F.seq = ++s->fin_seq;
        static const bool fin_clk = std::getenv("SVTGPU_LR_FIN_CLK") != nullptr;
        static unsigned long long *d_clk = nullptr;
        if (fin_clk && !d_clk) HIP_TRY(hipMalloc(&d_clk, 64));
        F.clk = fin_clk ? d_clk : nullptr;
        static const int fin_win = [] {
            const char *e = std::getenv("SVTGPU_LR_FIN_WIN");
            return e ? std::max(1, std::min(FIN_K1, std::atoi(e))) : FIN_K1;
        }();
        F.wtab = fin_win;
        if (tables) {
            hipLaunchKernelGGL(lr_fin_tables_kernel, dim3(F.pl[nplanes - 1].base + F.pl[nplanes - 1].n), dim3(64), 0,
                               st, F);
            HIP_TRY(hipGetLastError());
        }
        hipLaunchKernelGGL(lr_fin_walk_kernel, dim3(1), dim3(FIN_NT), 0, st, F);
        HIP_TRY(hipGetLastError());
        if (search_out) { // the records, all planes' units
            HIP_TRY(hipMemcpyAsync(hp(h_rec), dp(o_rec), sizeof(SvtGpuLrUnitSearch) * (size_t)nrec,
                                   hipMemcpyDeviceToHost, st));
            svtgpu_count_xfer(1, sizeof(SvtGpuLrUnitSearch) * (size_t)nrec);
        }
        if (!s->pin_free) HIP_TRY(hipEventCreateWithFlags(&s->pin_free, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->pin_free, st));
        s->fin_pending = 1;
        mark(3);
        if (!frame_type) return SVTGPU_OK; // asynchronous: svtgpu_lr_read_result collects the frame types
        if (int rc = lr_collect(s, st, frame_type)) return rc;
        if (F.clk) {
            unsigned long long v[8];
            HIP_TRY(hipMemcpy(v, F.clk, 64, hipMemcpyDeviceToHost));
            std::fprintf(stderr, "lr_fin_walk us: r1/r2 walks %.1f, switchable walks %.1f (luma: %llu chunks, preparation "
                                 "%.1f, steps %.1f), sums %.1f, types %.1f\n",
                         (v[1] - v[0]) * 0.01, (v[2] - v[1]) * 0.01, v[7], v[5] * 0.01, v[6] * 0.01, (v[3] - v[2]) * 0.01,
                         (v[4] - v[3]) * 0.01);
        }
        if (search_out) {
            const SvtGpuLrUnitSearch *hr = (const SvtGpuLrUnitSearch *)hp(h_rec);
            for (int p = 0; p < 3; p++)
                if (search_out[p]) std::memcpy(search_out[p], hr + rbase[p], sizeof(SvtGpuLrUnitSearch) * F.pl[p].n);
        }
        mark(4);
        if (timing)
            std::fprintf(stderr, "lr_search ms: stats+flt %.3f  seeds %.3f  descents %.3f  device finish + wait %.3f\n",
                         t_ph[0], t_ph[1], t_ph[2], t_ph[3] + t_ph[4]);
        return SVTGPU_OK;
    }
    Descent        *hw = (Descent *)hp(h_wds);
    const int32_t  *hbest = (const int32_t *)hp(h_best), *hraw = (const int32_t *)hp(h_braw);
    SvtGpuRestUnit *wu = (SvtGpuRestUnit *)hp(h_wu);
    HIP_TRY(hipMemcpyAsync(hp(h_res), dp(o_sse), res_span, hipMemcpyDeviceToHost, st)); // every result, one copy
    svtgpu_count_xfer(1, res_span);
    if (int rc = svtgpu_comm_wait(s->comm, st)) return rc; // bounded when an exchange sits before it
    if (n_wn && *(const int32_t *)hp(h_res + (o_wstat - o_sse))) { // status bits of wiener_res_kernel
        svtgpu_set_last_hip_error(hipErrorUnknown, "LR Wiener descent: round bound or part exchange timed out",
                                  __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    if (n_wr && wr_stat) {
        unsigned long long v[16];
        HIP_TRY(hipMemcpy(v, wr_stat, 128, hipMemcpyDeviceToHost));
        const double n = (double)std::max(1ull, v[0]), r = (double)std::max(1ull, v[1]);
        std::fprintf(stderr, "wiener_res: %llu items (%llu parted), %.1f candidates/item, %.0f px/item, per candidate: "
                     "%.2f us (thread 0: pass %.2f us, control %.2f us; wave passes: slowest %.2f us, fastest %.2f "
                     "us)\n", v[0], v[6], v[1] / n, v[5] / n, v[2] / r * 0.01, v[4] / r * 0.01, v[3] / r * 0.01,
                     v[7] / r * 0.01, v[8] / r * 0.01);
    }
    if (n_sr && sr_stat) {
        unsigned long long v[16];
        HIP_TRY(hipMemcpy(v, sr_stat, 128, hipMemcpyDeviceToHost));
        const double n = (double)std::max(1ull, v[0]);
        std::fprintf(stderr, "sgr_res: %llu items, %.2f passes/item, %.2f candidates/pass, %.0f px/item, ticks/item "
                     "load %.2f us, descent %.2f us (control %.2f us; pixel wave 0: passes %.2f us, waits B3-B4 %.2f "
                     "us; control wave before B3 %.2f us)\n", v[0], v[1] / n,
                     v[1] ? (double)v[2] / (double)v[6] * n / v[1] : 0.0, v[6] / n, v[3] / n * 0.01, v[4] / n * 0.01,
                     v[5] / n * 0.01, v[7] / n * 0.01, v[8] / n * 0.01, v[9] / n * 0.01);
        const double m = (double)std::max(1ull, v[10]), o = (double)std::max(1ull, v[0] - v[10]);
        std::fprintf(stderr, "sgr_res: row-part items %llu: load %.2f us, descent %.2f us (control %.2f us); one-part "
                     "items %llu: load %.2f us, descent %.2f us (control %.2f us)\n", v[10], v[11] / m * 0.01,
                     v[12] / m * 0.01, v[13] / m * 0.01, v[0] - v[10], (v[3] - v[11]) / o * 0.01,
                     (v[4] - v[12]) / o * 0.01, (v[5] - v[13]) / o * 0.01);
    }
    if (n_sr && *(const int32_t *)hp(h_res + (o_sstat - o_sse))) { // status bits of sgr_res_kernel
        svtgpu_set_last_hip_error(hipErrorUnknown, "LR self-guided descent: pass bound, part plan or exchange failed",
                                  __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    mark(3);
    // ---- phase 5 (host): per-unit results and, for the whole frame, the RD finish ----
    const uint64_t                 *sse0 = (const uint64_t *)hp(h_sse), *sse2 = (const uint64_t *)hp(h_sse2);
    SvtGpuRestUnit                 *out  = (SvtGpuRestUnit *)hp(h_out);
    std::vector<SvtGpuLrUnitSearch> rs(n_all);
    for (int p = 0; p < nplanes; p++) {
        const PlanePlan &q = pp[p];
        for (int u = 0; u < q.n; u++) {
            const int           gu = q.unit_base + u;
            SvtGpuLrUnitSearch &R  = rs[gu];
            std::memset(&R, 0, sizeof R);
            R.sse[0] = (int64_t)sse0[gu];
            R.sse[1] = INT64_MAX;
            if (q.wn && wu[gu].type) {
                R.sse[1] = hw[gu].err;
                R.wiener = wu[gu];
                int v[3];
                hw[gu].taps(0, v), set_wiener_taps(R.wiener.hfilter, v);
                hw[gu].taps(1, v), set_wiener_taps(R.wiener.vfilter, v);
            }
            if (q.sg) {
                const int bk = hbest[4 * gu]; // sgr_best_kernel: the first ep of least error
                R.sgrproj.type = SVTGPU_RESTORE_SGRPROJ, R.sgrproj.ep = q.eps[bk];
                R.sgrproj.xqd[0] = hraw[2 * gu], R.sgrproj.xqd[1] = hraw[2 * gu + 1];
                R.sse[2] = (int64_t)sse2[gu];
            }
            if (search_out && search_out[p]) search_out[p][uloc[gu]] = R;
        }
    }
    if (frame_type) { // whole frame: units are in plane order, uloc[gu] == u
        std::vector<FinRusi> rusi((size_t)std::max(1, pp[0].n));
        std::memset(rusi.data(), 0, sizeof(FinRusi) * rusi.size());
        for (int p = 0; p < nplanes; p++)
            finish_plane_shared(c, p, pp[p].win, rs.data() + pp[p].unit_base, pp[p].n, rusi.data(), &frame_type[p],
                                out + pp[p].unit_base);
    }
    if (frame_type) // d_units holds the planes back to back in the same order: one upload
        HIP_TRY(hipMemcpyAsync(s->d_units[0], out, sizeof(SvtGpuRestUnit) * n_all, hipMemcpyHostToDevice, st));
    if (frame_type) svtgpu_count_xfer(0, sizeof(SvtGpuRestUnit) * n_all);
    if (prof) { // algorithmic bytes per class (sample bytes bps, filter planes int16); the pixel-count parts at read
        const double bps = (double)sizeof(T);
        double       all = 0, wn = 0, sgb = 0, sgp = 0, sgw = 0; // sgw: filter planes written (equal r = 1 shared)
        for (int p = 0; p < nplanes; p++) {
            double area = 0;
            for (int i = pp[p].tile_base; i < pp[p].tile_base + pp[p].nt; i++) area += (double)tiles[i].w * tiles[i].h;
            all += area;
            if (pp[p].wn) wn += area;
            if (pp[p].sg) sgb += area, sgp += area * pp[p].ne;
            for (int k = 0; k < pp[p].ne; k++)
                sgw += area * ((kHostSgrR[A.pl[p].eps[k]][0] > 0) + (kHostSgrR[A.pl[p].eps[k]][1] > 0 && A.pl[p].f1e[k] == k));
        }
        prof->bps = bps;
        prof->static_bytes[0] += (all + wn) * 2 * bps; // unit sums, statistics: x and source
        prof->static_bytes[1] += sgb * bps + sgw * 2;     // filters: x in, the int16 planes out (each once)
        prof->static_bytes[3] += sgb * 2 * bps + sgp * 4; // resident search: x, source and every ep's planes, once
        prof->static_bytes[4] += sgb * (4 + 2 * bps);     // the chosen ep's SSE
    }
    // no wait for the units upload: the next search waits for this event before it rewrites the pinned staging
    if (!s->pin_free) HIP_TRY(hipEventCreateWithFlags(&s->pin_free, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(s->pin_free, st));
    mark(4);
    if (timing)
        std::fprintf(stderr, "lr_search ms: stats+flt %.3f  seeds %.3f  descents %.3f  best %.3f  finish %.3f\n",
                     t_ph[0], t_ph[1], t_ph[2], t_ph[3], t_ph[4]);
    return SVTGPU_OK;
}
} // namespace

int svtgpu_stats_unit_mfma8(int win, const uint8_t *dgd, const uint8_t *src, int h_start, int h_end, int v_start,
                            int v_end, int dgd_stride, int src_stride, int64_t *M, int64_t *H) {
    return stats_unit_mfma<uint8_t>(win, dgd, src, h_start, h_end, v_start, v_end, dgd_stride, src_stride, M, H, 1);
}
int svtgpu_stats_unit_mfma16(int win, const uint16_t *dgd, const uint16_t *src, int h_start, int h_end, int v_start,
                             int v_end, int dgd_stride, int src_stride, int64_t *M, int64_t *H, int div) {
    return stats_unit_mfma<uint16_t>(win, dgd, src, h_start, h_end, v_start, v_end, dgd_stride, src_stride, M, H, div);
}

extern "C" int svtgpu_lr_controls_for_level(int32_t wn, int32_t sg, SvtGpuLrSearchControls *c) {
    if (!c) return SVTGPU_ERR_INVALID_ARG;
    std::memset(c, 0, sizeof *c);
    // svt_aom_set_wn_filter_ctrls (EncModeConfig.c:1329-1384); level 6 reuses the previous frame's taps
    if (wn < 0 || wn > 5 || sg < 0 || sg > 4) return SVTGPU_ERR_UNSUPPORTED;
    if (wn > 0) {
        c->wn_enabled                 = 1;
        c->wn_use_chroma              = wn <= 4;
        c->wn_filter_tap_lvl          = wn <= 2 ? 1 : 2;
        c->wn_use_refinement          = wn <= 3;
        c->wn_max_one_refinement_step = wn >= 2;
    }
    // svt_aom_set_sg_filter_ctrls (EncModeConfig.c:1386-1445), fixed-range search (step_range 16)
    if (sg > 0) {
        c->sg_enabled     = 1;
        c->sg_use_chroma  = sg <= 3;
        c->sg_start_ep[0] = 0, c->sg_end_ep[0] = 16, c->sg_ep_inc[0] = sg >= 3 ? 8 : 1;
        c->sg_start_ep[1] = sg == 1 ? 0 : 4, c->sg_end_ep[1] = sg == 1 ? 16 : 5, c->sg_ep_inc[1] = 1;
        c->sg_refine[0] = 1, c->sg_refine[1] = sg == 1;
    }
    return SVTGPU_OK;
}

void lr_profiler_destroy(void *prof) { delete (LrProfiler *)prof; }

// the search's Wiener-chain stream (statistics, solve, ~48 trial rounds: the search's critical path) at the highest
// priority, so its workgroups are dispatched first while the self-guided filters fill the CUs.  Created with the
// state (svtgpu_lr_state_create), in the caller's order: a stream created lazily by the first search of each of
// several host threads landed on the hardware queues in thread order, and a queue shared with another frame's chain
// serializes the two (round 5's six-frames collapse)
int lr_make_wiener_stream(SvtGpuLrState *s) {
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    static const int wprio = [] { // SVTGPU_WN_PRIO=0: the Wiener chain at normal priority (A/B)
        const char *e = std::getenv("SVTGPU_WN_PRIO");
        return e ? std::atoi(e) : 1;
    }();
    HIP_TRY(hipStreamCreateWithPriority(&s->wst, hipStreamNonBlocking, wprio ? greatest : least));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_profile(SvtGpuLrState *s, int32_t enable, SvtGpuLrProfile *last) {
    if (!s) return SVTGPU_ERR_INVALID_ARG;
    LrProfiler *pr = (LrProfiler *)s->prof;
    if (last) {
        if (pr) {
            if (int rc = pr->read(last)) return rc;
        } else {
            std::memset(last, 0, sizeof *last);
        }
    }
    if (enable && !pr) {
        pr = new LrProfiler();
        if (!pr->ok) {
            delete pr;
            return SVTGPU_ERR_HIP;
        }
        s->prof = pr;
    }
    if (enable) {
        pr->mask   = enable < 0 ? 63 : enable & 63;
        pr->events = enable > 0 && (enable & 64);
        pr->serial = enable > 0 && (enable & 128);
    } else if (pr) {
        delete pr;
        s->prof = nullptr;
    }
    return SVTGPU_OK;
}

namespace {
int check_search_args(const SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                      const SvtGpuLrSearchControls *ctrls) {
    if (!s || !recon || !source || !ctrls || !lr_frame_fits(s, recon) || !lr_frame_fits(s, source) ||
        recon->bit_depth != source->bit_depth)
        return SVTGPU_ERR_INVALID_ARG;
    if (recon->bit_depth != 8 && recon->bit_depth != 10) return SVTGPU_ERR_UNSUPPORTED;
    for (int q = 0; q < 2; q++)
        if (ctrls->sg_enabled && (ctrls->sg_start_ep[q] < 0 || ctrls->sg_end_ep[q] > 16 || ctrls->sg_ep_inc[q] < 1))
            return SVTGPU_ERR_INVALID_ARG;
    return SVTGPU_OK;
}
int searched_planes(const SvtGpuLrSearchControls *c) {
    return ((c->wn_enabled && c->wn_use_chroma) || (c->sg_enabled && c->sg_use_chroma)) ? 3 : 1;
}
} // namespace

extern "C" int svtgpu_lr_search_frame(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                      const SvtGpuLrSearchControls *ctrls, int32_t frame_type_out[3],
                                      SvtGpuLrUnitSearch *const search_out[3], void *stream) {
    if (!frame_type_out) return SVTGPU_ERR_INVALID_ARG;
    if (int rc = check_search_args(s, recon, source, ctrls)) return rc;
    hipStream_t st      = pick_stream(s->ctx, stream);
    const int   nplanes = searched_planes(ctrls);
    for (int p = 0; p < 3; p++) frame_type_out[p] = SVTGPU_RESTORE_NONE;
    if (!lr_finish_on_host()) { // the records and the RD finish on the device; one wait at the end
        int32_t rb[3], re[3], cb[3], ce[3];
        for (int p = 0; p < 3; p++)
            cb[p] = s->tile_units[p][0], rb[p] = s->tile_units[p][1], ce[p] = s->tile_units[p][2], re[p] = s->tile_units[p][3];
        if (!svtgpu_comm_tiled(s->comm))
            for (int p = 0; p < 3; p++) rb[p] = cb[p] = 0, re[p] = s->vunits[p], ce[p] = s->hunits[p];
        return recon->bytes_per_sample == 2
            ? search_frame<uint16_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, frame_type_out, search_out, st, 1)
            : search_frame<uint8_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, frame_type_out, search_out, st, 1);
    }
    if (!svtgpu_comm_tiled(s->comm)) {
        int32_t rb[3] = {0, 0, 0}, re[3] = {s->vunits[0], s->vunits[1], s->vunits[2]};
        int32_t cb[3] = {0, 0, 0}, ce[3] = {s->hunits[0], s->hunits[1], s->hunits[2]};
        return recon->bytes_per_sample == 2
            ? search_frame<uint16_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, frame_type_out, search_out, st)
            : search_frame<uint8_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, frame_type_out, search_out, st);
    }
    // a picture tiled over GPUs: this rank's units, the zero-padded records summed over the ranks (one contributor per
    // unit: the gather restoration_seg_search's segments leave for rest_finish_search), then the finish of every
    // plane on every rank (EbRestorationPick.c:1555-1634, sequential over the units), identical everywhere
    size_t nrec = 0, base[3];
    for (int p = 0; p < 3; p++) base[p] = nrec, nrec += (size_t)s->hunits[p] * s->vunits[p];
    std::vector<SvtGpuLrUnitSearch> rec(nrec);
    std::memset(rec.data(), 0, sizeof(SvtGpuLrUnitSearch) * nrec);
    SvtGpuLrUnitSearch *outs[3] = {rec.data() + base[0], rec.data() + base[1], rec.data() + base[2]};
    int32_t             rb[3], re[3], cb[3], ce[3];
    for (int p = 0; p < 3; p++)
        cb[p] = s->tile_units[p][0], rb[p] = s->tile_units[p][1], ce[p] = s->tile_units[p][2], re[p] = s->tile_units[p][3];
    int rc = recon->bytes_per_sample == 2
        ? search_frame<uint16_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, nullptr, outs, st)
        : search_frame<uint8_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, nullptr, outs, st);
    if (rc) return rc;
    static_assert(sizeof(SvtGpuLrUnitSearch) % 8 == 0, "records travel as uint64 words");
    if ((rc = svtgpu_comm_sum(s->comm, rec.data(), nrec * sizeof(SvtGpuLrUnitSearch) / 8, false, st, SVTGPU_XCH_LR))) return rc;
    std::vector<SvtGpuRestUnit> units(nrec);
    std::memset(units.data(), 0, sizeof(SvtGpuRestUnit) * nrec);
    int32_t         nu[3];
    SvtGpuRestUnit *uo[3];
    for (int p = 0; p < 3; p++) nu[p] = s->hunits[p] * s->vunits[p], uo[p] = units.data() + base[p];
    finish_frame_host(ctrls, nplanes, nu, outs, frame_type_out, uo);
    for (int p = 0; p < nplanes; p++)
        if (search_out && search_out[p]) std::memcpy(search_out[p], outs[p], sizeof(SvtGpuLrUnitSearch) * nu[p]);
    HIP_TRY(hipMemcpyAsync(s->d_units[0], units.data(), sizeof(SvtGpuRestUnit) * nrec, hipMemcpyHostToDevice, st));
    svtgpu_count_xfer(0, sizeof(SvtGpuRestUnit) * nrec);
    if ((rc = svtgpu_comm_wait(s->comm, st))) return rc; // the host staging of the units goes out of scope
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_set_tile(SvtGpuLrState *s, const int32_t units[3][4], const int32_t out[3][4],
                                  SvtGpuComm *comm) {
    if (!s) return SVTGPU_ERR_INVALID_ARG;
    for (int p = 0; p < 3; p++) {
        const int pw = lr_plane_w(s, p), ph = lr_plane_h(s, p);
        const int32_t all_u[4] = {0, 0, s->hunits[p], s->vunits[p]}, all_o[4] = {0, 0, pw, ph};
        const int32_t *u = units ? units[p] : all_u, *o = out ? out[p] : all_o;
        if (u[0] < 0 || u[1] < 0 || u[2] > s->hunits[p] || u[3] > s->vunits[p] || u[0] > u[2] || u[1] > u[3])
            return SVTGPU_ERR_INVALID_ARG;
        // the output rect is a union of whole (stripe, 64 >> ss column) tiles of the apply
        const int S = 64 >> (p > 0), off = 8 >> (p > 0), cw = 64 >> (p > 0);
        auto row_ok = [&](int y) { return y == 0 || y == ph || (y + off) % S == 0; };
        auto col_ok = [&](int x) { return x == pw || x % cw == 0; };
        if (o[0] < 0 || o[1] < 0 || o[2] > pw || o[3] > ph || o[0] > o[2] || o[1] > o[3] || !col_ok(o[0]) ||
            !col_ok(o[2]) || !row_ok(o[1]) || !row_ok(o[3]))
            return SVTGPU_ERR_INVALID_ARG;
        std::memcpy(s->tile_units[p], u, sizeof s->tile_units[p]);
        std::memcpy(s->tile_out[p], o, sizeof s->tile_out[p]);
    }
    s->comm = comm;
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_search_units(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                      const SvtGpuLrSearchControls *ctrls, const int32_t row_begin[3],
                                      const int32_t row_end[3], SvtGpuLrUnitSearch *const search_out[3],
                                      void *stream) {
    if (!row_begin || !row_end || !search_out) return SVTGPU_ERR_INVALID_ARG;
    if (int rc = check_search_args(s, recon, source, ctrls)) return rc;
    const int nplanes = searched_planes(ctrls);
    for (int p = 0; p < nplanes; p++)
        if (row_begin[p] < 0 || row_end[p] > s->vunits[p] || row_begin[p] > row_end[p] || !search_out[p])
            return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    const int32_t cb[3] = {0, 0, 0}, ce[3] = {s->hunits[0], s->hunits[1], s->hunits[2]};
    return recon->bytes_per_sample == 2
        ? search_frame<uint16_t>(s, recon, source, ctrls, nplanes, row_begin, row_end, cb, ce, nullptr, search_out, st)
        : search_frame<uint8_t>(s, recon, source, ctrls, nplanes, row_begin, row_end, cb, ce, nullptr, search_out, st);
}

extern "C" int svtgpu_lr_finish_plane(const SvtGpuLrSearchControls *ctrls, int32_t plane, int32_t nunits,
                                      const SvtGpuLrUnitSearch *records, int32_t *frame_type_out,
                                      SvtGpuRestUnit *units_out) {
    if (!ctrls || plane < 0 || plane > 2 || nunits <= 0 || !records || !frame_type_out || !units_out)
        return SVTGPU_ERR_INVALID_ARG;
    for (int u = 0; u < nunits; u++) { // the rate helpers index tables with these fields
        const SvtGpuRestUnit &g = records[u].sgrproj;
        if (g.ep < 0 || g.ep > 15) return SVTGPU_ERR_INVALID_ARG;
    }
    if (plane >= searched_planes(ctrls)) {
        *frame_type_out = SVTGPU_RESTORE_NONE;
        std::memset(units_out, 0, sizeof(SvtGpuRestUnit) * nunits);
        return SVTGPU_OK;
    }
    // one plane alone: the shared array starts zeroed (a chroma plane's switchable pass sees no luma entries; the whole
    // frame's finish is svtgpu_lr_finish_frame)
    std::vector<FinRusi> rusi((size_t)nunits);
    std::memset(rusi.data(), 0, sizeof(FinRusi) * rusi.size());
    finish_plane_shared(ctrls, plane, plane_win(ctrls, plane), records, nunits, rusi.data(), frame_type_out, units_out);
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_finish_frame(const SvtGpuLrSearchControls *ctrls, const int32_t nunits[3],
                                      const SvtGpuLrUnitSearch *const records[3], int32_t frame_type_out[3],
                                      SvtGpuRestUnit *const units_out[3]) {
    if (!ctrls || !nunits || !records || !frame_type_out || !units_out) return SVTGPU_ERR_INVALID_ARG;
    const int nplanes = searched_planes(ctrls);
    for (int p = 0; p < 3; p++) {
        if (p >= nplanes) continue;
        if (nunits[p] <= 0 || !records[p] || !units_out[p] || (p && nunits[p] > nunits[0])) return SVTGPU_ERR_INVALID_ARG;
        for (int u = 0; u < nunits[p]; u++)
            if (records[p][u].sgrproj.ep < 0 || records[p][u].sgrproj.ep > 15) return SVTGPU_ERR_INVALID_ARG;
    }
    for (int p = 0; p < 3; p++) {
        frame_type_out[p] = SVTGPU_RESTORE_NONE;
        if (p >= nplanes && units_out[p] && nunits[p] > 0) std::memset(units_out[p], 0, sizeof(SvtGpuRestUnit) * nunits[p]);
    }
    finish_frame_host(ctrls, nplanes, nunits, records, frame_type_out, units_out);
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_search_frame_async(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                            const SvtGpuLrSearchControls *ctrls, void *stream) {
    if (int rc = check_search_args(s, recon, source, ctrls)) return rc;
    hipStream_t st      = pick_stream(s->ctx, stream);
    const int   nplanes = searched_planes(ctrls);
    if (lr_finish_on_host()) { // the host finish waits anyway: the synchronous search, its frame types kept
        int32_t ft[3];
        if (int rc = svtgpu_lr_search_frame(s, recon, source, ctrls, ft, nullptr, stream)) return rc;
        for (int p = 0; p < 3; p++) s->last_ft[p] = ft[p];
        s->fin_pending = 0;
        return SVTGPU_OK;
    }
    int32_t rb[3], re[3], cb[3], ce[3];
    for (int p = 0; p < 3; p++)
        cb[p] = s->tile_units[p][0], rb[p] = s->tile_units[p][1], ce[p] = s->tile_units[p][2], re[p] = s->tile_units[p][3];
    if (!svtgpu_comm_tiled(s->comm))
        for (int p = 0; p < 3; p++) rb[p] = cb[p] = 0, re[p] = s->vunits[p], ce[p] = s->hunits[p];
    return recon->bytes_per_sample == 2
        ? search_frame<uint16_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, nullptr, nullptr, st, 1)
        : search_frame<uint8_t>(s, recon, source, ctrls, nplanes, rb, re, cb, ce, nullptr, nullptr, st, 1);
}

extern "C" int svtgpu_lr_read_units(SvtGpuLrState *s, int32_t plane, SvtGpuRestUnit *units_out, void *stream) {
    if (!s || plane < 0 || plane > 2 || !units_out) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    if (s->fin_pending)
        if (int rc = lr_collect(s, st, nullptr)) return rc;
    const size_t n = (size_t)s->hunits[plane] * s->vunits[plane];
    HIP_TRY(hipMemcpyAsync(units_out, s->d_units[plane], sizeof(SvtGpuRestUnit) * n, hipMemcpyDeviceToHost, st));
    svtgpu_count_xfer(1, sizeof(SvtGpuRestUnit) * n);
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_read_result(SvtGpuLrState *s, int32_t frame_type_out[3], void *stream) {
    if (!s || !frame_type_out) return SVTGPU_ERR_INVALID_ARG;
    if (s->fin_pending) return lr_collect(s, pick_stream(s->ctx, stream), frame_type_out);
    for (int p = 0; p < 3; p++) frame_type_out[p] = s->last_ft[p];
    return SVTGPU_OK;
}
