// cdef_search.hip — fused CDEF strength search for whole frames (SB64), gfx950.
//
// ≙ cdef_seg_search over all segments (Source/Lib/Encoder/Codec/EbCdefProcess.c:114-357):
// for every 64x64 filter block (FB), every plane and every candidate strength, filter the listed
// 8x8 (luma) / 4x4 (chroma) blocks (svt_cdef_filter_fb, EbCdef.c:339) and measure the distortion
// against the source (compute_cdef_dist, EbCdefProcess.c:87 → EbEncCdef.c:129/175).
//
// One workgroup (256 lanes) per FB; the DLF-output tile (+-2 px context, 0x7F7F outside the frame —
// exactly the samples the reference stages, EbCdefProcess.c:206-236) lives in LDS.
//
// Work decomposition (the reason this is fast): the filter output is
//     y = clamp(x + round(P(pri) + S(sec)), lo, hi)
// where P sums the 4 primary taps (depends only on the primary strength, adjusted per block) and S
// the 8 secondary taps (depends only on the secondary strength); lo/hi depend on neither (EbCdef.c:
// 263-297; int16 sums never wrap for 8/10-bit input).  So per tap-direction set each lane evaluates
// S once per secondary strength (3) and P once per primary level (<= 16) — 16x4 + 3x8 tap
// constraints instead of 64x12 — and each of the 64 strengths costs only the rounding, clamp and
// distortion statistics.  Everything is packed int16 (two samples per VGPR).
// Lanes own whole rows of 8 samples (4 pairs): a luma 8x8 block is 8 lanes, so its per-strength
// statistics (sum d, sum d^2, sum (d-s)^2) reduce with 3 DPP steps; the double-precision SSIM-like
// distortion (EbEncCdef.c:42-47) runs once per (strength, block) in a lane-parallel epilogue.
#include "cdef_common.h"

#define NT 256
#define LT 70 // luma tile row stride (68 columns -2..65 used): an odd dword stride spreads a wave's rows over the LDS banks
#define CT 38 // chroma tile row stride (36 columns used), odd in dwords likewise

struct SearchArgs {
    const void    *rec[3];
    const void    *src[3];
    int32_t        rstride[3], sstride[3];
    int32_t        width, height;
    int32_t        b8_cols, nhfb;
    const uint8_t *mask;
    uint64_t      *mse;  // [2][nfb][64]
    uint8_t       *skip; // [nfb]
    uint8_t       *dir;  // [nfb][64]
    int32_t       *var;  // [nfb][64]
    uint8_t       *rem;  // [3][nfb][64] low 2*cs bits of the luma / Cb / Cr sums before the shift, or null
    int32_t        nfb, fb0, fbw; // searched filter blocks: fb0 + (i / fbw) * nhfb + i % fbw
    int32_t        cs, ss, damping;
    CdefStrengthTable tab;
    unsigned long long *wgclk; // diagnostics (svtgpu_internal.h wgclk_mark) or null
};

struct PriPair { // two horizontally adjacent samples, packed int16 (lo half = left sample)
    s16x2 x, lo, hi;
    s16x2 d[4]; // p - x of the primary taps: (k0,+), (k0,-), (k1,+), (k1,-) (the magnitude is formed per use: fewer
                // live registers, so the kernel holds three waves per SIMD)
};

// 8 samples from an 8-aligned position of a plane as four packed int16 pairs (one 16-B / 8-B load)
template <typename T>
__device__ __forceinline__ void ld_seg8(const void *base, long idx, s16x2 out[4]) {
    const T *p = (const T *)base + idx;
    if constexpr (sizeof(T) == 2) {
        const uint4 w = *(const uint4 *)p;
        out[0] = __builtin_bit_cast(s16x2, w.x), out[1] = __builtin_bit_cast(s16x2, w.y);
        out[2] = __builtin_bit_cast(s16x2, w.z), out[3] = __builtin_bit_cast(s16x2, w.w);
    } else {
        const uint2 b = *(const uint2 *)p;
        out[0] = __builtin_bit_cast(s16x2, (b.x & 0xFF) | ((b.x & 0xFF00) << 8));
        out[1] = __builtin_bit_cast(s16x2, ((b.x >> 16) & 0xFF) | ((b.x >> 8) & 0xFF0000));
        out[2] = __builtin_bit_cast(s16x2, (b.y & 0xFF) | ((b.y & 0xFF00) << 8));
        out[3] = __builtin_bit_cast(s16x2, ((b.y >> 16) & 0xFF) | ((b.y >> 8) & 0xFF0000));
    }
}

// Stage a plane tile (rows r0-2 .. r0+n+1, cols c0-2 .. c0+n+1) into LDS, 0x7F7F outside the plane: every interior
// 8-sample row segment one vector load (all of a lane's loads in flight before the first LDS store) and four 4-B LDS
// stores (the tile rows keep the bank-spreading stride TS; the interior starts at column 2), the apron one sample each.
// The rows are padded to 256 B, so a segment that starts inside the plane reads only its own row.
template <typename T, int N, int TS>
__device__ __forceinline__ void stage_tile(uint16_t *tile, const void *plane_, int stride, int pw, int ph, int r0,
                                           int c0) {
    const T      *plane = (const T *)plane_;
    constexpr int ROWS = N + 2 * CDEF_BORDER, SEGS = N / 8, NI = ROWS * SEGS, IT = (NI + NT - 1) / NT;
    constexpr int NB = ROWS * 4, IB = (NB + NT - 1) / NT;
    uint4         v[IT];
#pragma unroll
    for (int u = 0; u < IT; u++) {
        const int i = threadIdx.x + u * NT, r = i / SEGS, sg = i % SEGS;
        const int fr = r0 + r - CDEF_BORDER, fc = c0 + 8 * sg;
        v[u] = (uint4){0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu};
        if (i >= NI || fr < 0 || fr >= ph || fc >= pw) continue;
        const T *src = plane + (long)fr * stride + fc;
        if constexpr (sizeof(T) == 2) {
            v[u] = *(const uint4 *)src;
        } else {
            const uint2 b = *(const uint2 *)src;
            v[u] = (uint4){(b.x & 0xFF) | ((b.x & 0xFF00) << 8), ((b.x >> 16) & 0xFF) | ((b.x >> 8) & 0xFF0000),
                           (b.y & 0xFF) | ((b.y & 0xFF00) << 8), ((b.y >> 16) & 0xFF) | ((b.y >> 8) & 0xFF0000)};
        }
        if (fc + 8 > pw) { // the plane's last segment of a row (chroma widths of 4 mod 8)
            uint32_t *q = &v[u].x;
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (fc + j >= pw) q[j >> 1] = (j & 1) ? (q[j >> 1] & 0xFFFFu) | 0x7F7F0000u : (q[j >> 1] & 0xFFFF0000u) | 0x7F7Fu;
        }
    }
    uint16_t b[IB];
#pragma unroll
    for (int u = 0; u < IB; u++) {
        const int i = threadIdx.x + u * NT, r = i >> 2, k = i & 3, dc = k < 2 ? k - 2 : N + k - 2;
        const int fr = r0 + r - CDEF_BORDER, fc = c0 + dc;
        b[u] = CDEF_VERY_LARGE_V;
        if (i < NB && fr >= 0 && fr < ph && fc >= 0 && fc < pw) b[u] = (uint16_t)plane[(long)fr * stride + fc];
    }
#pragma unroll
    for (int u = 0; u < IT; u++) {
        const int i = threadIdx.x + u * NT, r = i / SEGS, sg = i % SEGS;
        if (i >= NI) continue;
        uint32_t *d = (uint32_t *)(tile + r * TS + CDEF_BORDER + 8 * sg); // 4-B aligned: TS and the offset are even
        d[0] = v[u].x, d[1] = v[u].y, d[2] = v[u].z, d[3] = v[u].w;
    }
#pragma unroll
    for (int u = 0; u < IB; u++) {
        const int i = threadIdx.x + u * NT, r = i >> 2, k = i & 3, dc = k < 2 ? k - 2 : N + k - 2;
        if (i < NB) tile[r * TS + CDEF_BORDER + dc] = b[u];
    }
}

__device__ __forceinline__ s16x2 splat16(int v) { return (s16x2){(short)v, (short)v}; }
__device__ __forceinline__ u16x2 splatu16(int v) { return (u16x2){(unsigned short)v, (unsigned short)v}; }

// constrain(d, thr, damping) = sign(d) * min(|d|, m), m = max(0, thr - (|d| >> shift)) (EbCdef.c:85-91): m >= 0, so it
// is the clamp of d to [-m, m]
__device__ __forceinline__ s16x2 constrain2(s16x2 d, s16x2 thr, u16x2 sh) {
    const s16x2 ad = __builtin_elementwise_max(d, (s16x2){0, 0} - d);
    const s16x2 m  = __builtin_elementwise_max(thr - (s16x2)(((u16x2)ad) >> sh), (s16x2){0, 0});
    return __builtin_elementwise_max(__builtin_elementwise_min(d, m), (s16x2){0, 0} - m);
}

// Neighbourhood of the pair at tile (r, c), (r, c+1) for direction `dir`: keeps the primary taps
// and the clamp range, and returns the secondary sums S[1..3] for the secondary codes in `sec_used`.
// The pair of samples at 16-bit index a of an LDS tile from two aligned dwords (one ds_read2_b32) and a funnel
// shift: a dword read at an odd sample index is a misaligned LDS access, which the LDS serves far below its rate.
__device__ __forceinline__ uint32_t lds_pair_u32(const uint16_t *tile, int a) {
    const uint32_t *w = (const uint32_t *)tile + (a >> 1);
    return __builtin_amdgcn_alignbit(w[1], w[0], (a & 1) * 16);
}

__device__ __forceinline__ void load_pair(PriPair &P, s16x2 S[4], const uint16_t *tile, int ts, int r, int c,
                                          int dir, int sec_used, int sdamp, int cs) {
    const int       a0 = (r + CDEF_BORDER) * ts + (c + CDEF_BORDER); // even: ts and c are
    const uint32_t  xw = *(const uint32_t *)(tile + a0);
    const int       xa = (int16_t)(xw & 0xFFFF), xb = (int16_t)(xw >> 16);
    int             loa = xa, hia = xa, lob = xb, hib = xb;
    const int       ds0 = (dir + 2) & 7, ds1 = (dir + 6) & 7;
    s16x2           sd[8];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int op = cdef_dir_dy(dir, k) * ts + cdef_dir_dx(dir, k);
        const int o0 = cdef_dir_dy(ds0, k) * ts + cdef_dir_dx(ds0, k);
        const int o1 = cdef_dir_dy(ds1, k) * ts + cdef_dir_dx(ds1, k);
        const int o[6] = {op, -op, o0, -o0, o1, -o1};
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const uint32_t vw = lds_pair_u32(tile, a0 + o[t]);
            const int      va = (int16_t)(vw & 0xFFFF), vb = (int16_t)(vw >> 16);
            if (va != CDEF_VERY_LARGE_V) hia = max(hia, va);
            if (vb != CDEF_VERY_LARGE_V) hib = max(hib, vb);
            loa = min(loa, va);
            lob = min(lob, vb);
            const s16x2 dd = {(short)(va - xa), (short)(vb - xb)};
            if (t < 2)
                P.d[2 * k + t] = dd;
            else
                sd[4 * k + t - 2] = dd;
        }
    }
    P.x  = (s16x2){(short)xa, (short)xb};
    P.lo = (s16x2){(short)loa, (short)lob};
    P.hi = (s16x2){(short)hia, (short)hib};
    S[0] = (s16x2){0, 0};
#pragma unroll
    for (int sc = 1; sc < 4; sc++) {
        S[sc] = (s16x2){0, 0};
        if (!(sec_used & (1 << sc))) continue; // workgroup-uniform
        const int   sec = (sc == 3 ? 4 : sc) << cs;
        const s16x2 thr = splat16(sec);
        const u16x2 sh  = splatu16(max(0, sdamp - msb32_dev((uint32_t)sec)));
        s16x2       a0 = {0, 0}, a1 = {0, 0};
#pragma unroll
        for (int t = 0; t < 4; t++) {
            a0 = a0 + constrain2(sd[t], thr, sh);     // k = 0, tap weight 2
            a1 = a1 + constrain2(sd[4 + t], thr, sh); // k = 1, tap weight 1
        }
        S[sc] = (a0 << (s16x2){1, 1}) + a1;
    }
}

// primary sum for threshold `thr` (already strength-adjusted), weights {4,2} or {3,3}
__device__ __forceinline__ s16x2 pri_sum(const PriPair &P, s16x2 thr, u16x2 sh, s16x2 w0, s16x2 w1) {
    const s16x2 k0 = constrain2(P.d[0], thr, sh) + constrain2(P.d[1], thr, sh);
    const s16x2 k1 = constrain2(P.d[2], thr, sh) + constrain2(P.d[3], thr, sh);
    return k0 * w0 + k1 * w1;
}

// y = clamp(x + ((8 + sum - (sum < 0)) >> 4), lo, hi)   (EbCdef.c:298)
__device__ __forceinline__ s16x2 finish(const PriPair &P, s16x2 sum) {
    const s16x2 rnd = (sum + (s16x2){8, 8} + (sum >> (s16x2){15, 15})) >> (s16x2){4, 4};
    return __builtin_elementwise_max(__builtin_elementwise_min(P.x + rnd, P.hi), P.lo);
}

// sum over the 8 lanes of each aligned octet (quad xor1, quad xor2, row_half_mirror)
__device__ __forceinline__ uint32_t oct_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    return v;
}

template <typename T>
__global__ void __launch_bounds__(NT, 3) cdef_search_kernel(const SearchArgs A) {
    __shared__ __attribute__((aligned(16))) uint16_t ltile[(64 + 2 * CDEF_BORDER) * LT];
    __shared__ __attribute__((aligned(16))) uint16_t ctile[2][(32 + 2 * CDEF_BORDER) * CT];
    __shared__ uint32_t stats[64][32][3]; // per pass: [gi][block-in-pass][sum_d, sum_d2, sse]
    __shared__ uint32_t sstat[64][2];     // per block source sum, sum^2 (luma)
    __shared__ uint64_t acc_l[64];        // per gi luma distortion
    __shared__ uint32_t acc_c[2][64];     // per gi chroma SSE per plane
    __shared__ int32_t  dcost[64][8];
    __shared__ uint8_t  sdir[64];
    __shared__ int32_t  svar[64];
    __shared__ uint8_t  slisted[64];
    __shared__ int32_t  nlisted;
    __shared__ CdefGroupTable grp[4]; // luma A, luma B, chroma A, chroma B

    wgclk_mark(A.wgclk, 0);
    const int fi = xcd_swizzle(blockIdx.x, gridDim.x), fb = A.fb0 + (fi / A.fbw) * A.nhfb + fi % A.fbw;
    const int fbr = fb / A.nhfb, fbc = fb - fbr * A.nhfb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cs = A.cs;

    // ---- block list (svt_sb_compute_cdef_list, EbEncCdef.c:238-282) + strength tables ----
    if (tid == 0) nlisted = 0;
    {
        const int32_t *src = (const int32_t *)&A.tab.luma[0];
        int32_t       *dst = (int32_t *)&grp[0];
        for (int i = tid; i < (int)(sizeof(grp) / 4); i += NT) dst[i] = src[i];
    }
    __syncthreads();
    if (tid < 64) {
        const int by = tid >> 3, bx = tid & 7;
        const int br = 8 * fbr + by, bc = 8 * fbc + bx;
        const int in_frame = (8 * br < A.height) && (8 * bc < A.width);
        const int l = in_frame && (A.mask ? A.mask[br * A.b8_cols + bc] : 1);
        slisted[tid] = (uint8_t)l;
        if (l) atomicAdd(&nlisted, 1);
        acc_l[tid]    = 0;
        acc_c[0][tid] = 0;
        acc_c[1][tid] = 0;
    }
    __syncthreads();
    if (nlisted == 0) { // EbCdefProcess.c:209-212
        if (tid == 0) A.skip[fb] = 1;
        if (tid < 64) {
            A.mse[(size_t)fb * 64 + tid]           = 0;
            A.mse[((size_t)A.nfb + fb) * 64 + tid] = 0;
            if (A.rem)
                for (int k = 0; k < 3; k++) A.rem[((size_t)k * A.nfb + fb) * 64 + tid] = 0;
            A.dir[(size_t)fb * 64 + tid]           = 0;
            A.var[(size_t)fb * 64 + tid]           = 0;
        }
        return;
    }

    wgclk_mark(A.wgclk, 1);
    // ---- stage tiles ----
    stage_tile<T, 64, LT>(ltile, A.rec[0], A.rstride[0], A.width, A.height, 64 * fbr, 64 * fbc);
    stage_tile<T, 32, CT>(ctile[0], A.rec[1], A.rstride[1], A.width >> 1, A.height >> 1, 32 * fbr, 32 * fbc);
    stage_tile<T, 32, CT>(ctile[1], A.rec[2], A.rstride[2], A.width >> 1, A.height >> 1, 32 * fbr, 32 * fbc);
    __syncthreads();

    wgclk_mark(A.wgclk, 2);
    // ---- direction per 8x8 luma block (svt_aom_cdef_find_dir_c, EbCdef.c:150-210) ----
    // wave w computes directions 2w and 2w+1 for block = lane (direction wave-uniform); the block's rows are read
    // from LDS inside each direction's accumulation (4 dword reads per row) instead of being held in 64 registers
    {
        const int b = lane, by = b >> 3, bx = b & 7;
        const int w840[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
        const uint16_t *blk = ltile + (8 * by + CDEF_BORDER) * LT + 8 * bx + CDEF_BORDER; // 4-B aligned
#pragma unroll
        for (int dd = 0; dd < 2; dd++) {
            const int d = 2 * wave + dd;
            int       line[15];
#pragma unroll
            for (int k = 0; k < 15; k++) line[k] = 0;
            int cost = 0;
            switch (d) { // partial-sum line of sample (i, j) per direction (EbCdef.c:171-179)
#define ACC(EXPR)                                                                                              \
    _Pragma("unroll") for (int i = 0; i < 8; i++) {                                                            \
        const uint32_t *rw = (const uint32_t *)(blk + i * LT);                                                 \
        const uint32_t  w[4] = {rw[0], rw[1], rw[2], rw[3]};                                                   \
        _Pragma("unroll") for (int j = 0; j < 8; j++) line[EXPR] += (int)((w[j >> 1] >> (16 * (j & 1)) & 0xFFFFu) >> cs) - 128; \
    }
            case 0: ACC(i + j) break;
            case 1: ACC(i + j / 2) break;
            case 2: ACC(i) break;
            case 3: ACC(3 + i - j / 2) break;
            case 4: ACC(7 + i - j) break;
            case 5: ACC(3 - i / 2 + j) break;
            case 6: ACC(j) break;
            default: ACC(i / 2 + j) break;
#undef ACC
            }
            if (d == 2 || d == 6) {
#pragma unroll
                for (int k = 0; k < 8; k++) cost += line[k] * line[k];
                cost *= w840[8];
            } else if (d == 0 || d == 4) {
                cost = line[7] * line[7] * w840[8];
#pragma unroll
                for (int k = 0; k < 7; k++) cost += (line[k] * line[k] + line[14 - k] * line[14 - k]) * w840[k + 1];
            } else {
#pragma unroll
                for (int k = 3; k < 8; k++) cost += line[k] * line[k];
                cost *= w840[8];
#pragma unroll
                for (int k = 0; k < 3; k++) cost += (line[k] * line[k] + line[10 - k] * line[10 - k]) * w840[2 * k + 2];
            }
            dcost[b][d] = cost;
        }
    }
    __syncthreads();
    if (tid < 64) {
        int best = 0, bd = 0;
#pragma unroll
        for (int d = 0; d < 8; d++)
            if (dcost[tid][d] > best) {
                best = dcost[tid][d];
                bd   = d;
            }
        const int v = (best - dcost[tid][(bd + 4) & 7]) >> 10;
        sdir[tid]   = (uint8_t)bd;
        svar[tid]   = v;
        A.dir[(size_t)fb * 64 + tid] = (uint8_t)bd;
        A.var[(size_t)fb * 64 + tid] = v;
    }
    __syncthreads();

    const int ldamp = A.damping + cs, cdamp = A.damping + cs - 1;
    const int ss    = A.ss;
    const int nstr  = A.tab.nstr;

    wgclk_mark(A.wgclk, 3);
    // ================= luma: 2 passes of 32 blocks; lane = one 8-sample row =================
    for (int pass = 0; pass < 2; pass++) {
        // block in pass, row in block.  A wave holds one row of 8 blocks; its lower half the even block columns, its
        // upper half the odd ones: the half-wave's rows then sit at 35 r + 8 j dwords (r < 8, j < 4), 32 distinct
        // banks for every tap read (with the 4 adjacent blocks of a half, (r, j) and (r + 4, j + 3) shared a bank)
        const int bip = ((tid >> 6) << 3) | (((tid >> 3) & 3) << 1) | ((tid >> 5) & 1), row = tid & 7;
        const int b = 32 * pass + bip, by = b >> 3, bx = b & 7;
        const int r = 8 * by + row, c0 = 8 * bx;
        const bool valid = slisted[b] && (row % ss == 0);
        const unsigned short vm = valid ? 0xFFFF : 0;
        // source row (registers), zeroed outside the measured set
        s16x2 sp[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        if (valid) ld_seg8<T>(A.src[0], (long)(64 * fbr + r) * A.sstride[0] + 64 * fbc + c0, sp);
        {
            uint32_t s1 = 0, s2 = 0;
#pragma unroll
            for (int h = 0; h < 4; h++) {
                s1 = __builtin_amdgcn_udot2((u16x2)sp[h], (u16x2){1, 1}, s1, false);
                s2 = __builtin_amdgcn_udot2((u16x2)sp[h], (u16x2)sp[h], s2, false);
            }
            s1 = oct_sum(s1);
            s2 = oct_sum(s2);
            if (row == 0) {
                sstat[b][0] = s1;
                sstat[b][1] = s2;
            }
        }
        const int vb = svar[b];
        const int ib = (vb >> 6) ? min(msb32_dev((uint32_t)(vb >> 6)), 12) : 0;
        for (int g = 0; g < 2; g++) {
            const CdefGroupTable &G = grp[g];
            if (G.nlv == 0) continue;
            const int d = g ? sdir[b] : 0; // pri_strength ? dir : 0 (EbCdef.c:404)
            PriPair   P[4];
            s16x2     S[4][4];
#pragma unroll
            for (int h = 0; h < 4; h++) load_pair(P[h], S[h], ltile, LT, r, c0 + 2 * h, d, G.sec_used, ldamp, cs);
            for (int li = 0; li < G.nlv; li++) {
                const int pri = G.lv[li] << cs;
                const int t   = vb ? (pri * (4 + ib) + 8) >> 4 : 0; // adjust_strength (EbCdef.c:130-135)
                const int odd = (t >> cs) & 1;
                const s16x2 thr = splat16(t);
                const u16x2 sh  = splatu16(max(0, ldamp - msb32_dev((uint32_t)t)));
                const s16x2 w0 = splat16(odd ? 3 : 4), w1 = splat16(odd ? 3 : 2);
                s16x2 Pv[4];
#pragma unroll
                for (int h = 0; h < 4; h++) Pv[h] = pri_sum(P[h], thr, sh, w0, w1);
#pragma unroll
                for (int sc = 0; sc < 4; sc++) {
                    const int gi = G.gi[li][sc];
                    if (gi < 0) continue; // workgroup-uniform
                    uint32_t sd = 0, sd2 = 0, sse = 0;
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        s16x2 y = finish(P[h], Pv[h] + S[h][sc]);
                        y       = (s16x2)((u16x2)y & (u16x2){vm, vm});
                        const s16x2 df = y - sp[h];
                        sd  = __builtin_amdgcn_udot2((u16x2)y, (u16x2){1, 1}, sd, false);
                        sd2 = __builtin_amdgcn_udot2((u16x2)y, (u16x2)y, sd2, false);
                        sse = (uint32_t)__builtin_amdgcn_sdot2(df, df, (int)sse, false);
                    }
                    sd  = oct_sum(sd);
                    sd2 = oct_sum(sd2);
                    sse = oct_sum(sse);
                    if (row == 0) {
                        stats[gi][bip][0] = sd;
                        stats[gi][bip][1] = sd2;
                        stats[gi][bip][2] = sse;
                    }
                }
            }
        }
        __syncthreads();
        // double-precision distortion per (gi, block): 4 lanes per gi, 8 blocks per lane
        {
            const int gi = tid >> 2, sub = tid & 3;
            unsigned long long acc = 0;
            if (gi < nstr && A.tab.alias[gi] < 0) {
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int bb = 8 * sub + u, bg = 32 * pass + bb;
                    if (!slisted[bg]) continue;
                    acc += cdef_luma_dist(stats[gi][bb][0], sstat[bg][0], stats[gi][bb][1], sstat[bg][1],
                                          stats[gi][bb][2], cs);
                }
            }
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            if (sub == 0 && gi < nstr) acc_l[gi] += acc;
        }
        __syncthreads();
    }

    wgclk_mark(A.wgclk, 4);
    // ================= chroma: both planes in one pass; lane = one 8-sample row =================
    {
        // plane, row, segment.  A half-wave holds rows {4h .. 4h + 3, 4h + 16 .. 4h + 19} (h < 4) and the 4 segments of
        // each: at the 19-dword row stride those are 32 distinct banks (8 consecutive rows shared 4 of them pairwise)
        const int pl = tid >> 7, q = tid & 127, hq = q >> 5, rr = (q >> 2) & 7;
        const int r = 4 * hq + (rr & 3) + 16 * (rr >> 2), c0 = (q & 3) * 8;
        const int by = r >> 2;
        const uint16_t *tile = ctile[pl];
        s16x2 sp[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        unsigned short vm[4];
        int  dirb[4];
        const int cb0 = by * 8 + (c0 >> 2); // the segment's two 4x4 chroma blocks: cb0, cb0 + 1
        if (slisted[cb0] || slisted[cb0 + 1]) // inside the plane: listed blocks are in the frame, widths are even
            ld_seg8<T>(A.src[1 + pl], (long)(32 * fbr + r) * A.sstride[1 + pl] + 32 * fbc + c0, sp);
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int cb = cb0 + (h >> 1);
            vm[h]   = slisted[cb] ? 0xFFFF : 0;
            dirb[h] = sdir[cb];
            if (!slisted[cb]) sp[h] = (s16x2){0, 0};
        }
        for (int g = 0; g < 2; g++) {
            const CdefGroupTable &G = grp[2 + g];
            if (G.nlv == 0) continue;
            PriPair P[4];
            s16x2   S[4][4];
#pragma unroll
            for (int h = 0; h < 4; h++)
                load_pair(P[h], S[h], tile, CT, r, c0 + 2 * h, g ? dirb[h] : 0, G.sec_used, cdamp, cs);
            for (int li = 0; li < G.nlv; li++) {
                const int pri = G.lv[li] << cs; // no strength adjustment for chroma (EbCdef.c:401)
                const int odd = (pri >> cs) & 1;
                const s16x2 thr = splat16(pri);
                const u16x2 sh  = splatu16(max(0, cdamp - msb32_dev((uint32_t)pri)));
                const s16x2 w0 = splat16(odd ? 3 : 4), w1 = splat16(odd ? 3 : 2);
                s16x2 Pv[4];
#pragma unroll
                for (int h = 0; h < 4; h++) Pv[h] = pri_sum(P[h], thr, sh, w0, w1);
#pragma unroll
                for (int sc = 0; sc < 4; sc++) {
                    const int gi = G.gi[li][sc];
                    if (gi < 0) continue;
                    uint32_t sse = 0;
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        s16x2 y = finish(P[h], Pv[h] + S[h][sc]);
                        y       = (s16x2)((u16x2)y & (u16x2){vm[h], vm[h]});
                        const s16x2 df = y - sp[h];
                        sse = (uint32_t)__builtin_amdgcn_sdot2(df, df, (int)sse, false);
                    }
                    sse = row16_sum(sse);
                    if ((lane & 15) == 0) atomicAdd(&acc_c[pl][gi], sse);
                }
            }
        }
    }
    __syncthreads();

    // ---- per-FB mse rows (EbCdefProcess.c:293-298, :349-353) ----
    if (tid < 64) {
        const int gi = tid;
        uint64_t  m0 = 0, m1 = 0;
        if (gi < nstr) {
            const int src = A.tab.alias[gi] < 0 ? gi : A.tab.alias[gi];
            m0 = (acc_l[src] >> (2 * cs)) * (uint64_t)ss;
            m1 = A.tab.uv_on[gi] ? ((uint64_t)(acc_c[0][src] >> (2 * cs)) + (uint64_t)(acc_c[1][src] >> (2 * cs)))
                                 : 1040400ull * 64; // default_mse_uv * 64
        }
        A.mse[(size_t)fb * 64 + gi]           = m0;
        A.mse[((size_t)A.nfb + fb) * 64 + gi] = m1;
        if (A.rem) { // what the shift drops: a 128-wide SB128 area shifts the sum of its parts (cdef_sb128.hip)
            const int      src  = gi < nstr && A.tab.alias[gi] >= 0 ? A.tab.alias[gi] : gi;
            const uint32_t mask = (1u << (2 * cs)) - 1;
            const bool     on   = gi < nstr;
            A.rem[(size_t)fb * 64 + gi]                   = on ? (uint8_t)(acc_l[src] & mask) : 0;
            A.rem[((size_t)A.nfb + fb) * 64 + gi]         = on && A.tab.uv_on[gi] ? (uint8_t)(acc_c[0][src] & mask) : 0;
            A.rem[((size_t)2 * A.nfb + fb) * 64 + gi]     = on && A.tab.uv_on[gi] ? (uint8_t)(acc_c[1][src] & mask) : 0;
        }
        if (tid == 0) A.skip[fb] = 0;
    }
    wgclk_mark(A.wgclk, 5);
}

int svtgpu_launch_cdef_search(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, const SvtGpuFrame *src,
                              const CdefStrengthTable *tab, int32_t subsampling, int32_t damping, hipStream_t st) {
    SearchArgs A;
    for (int p = 0; p < 3; p++) {
        A.rec[p]     = recon->plane[p];
        A.src[p]     = src->plane[p];
        A.rstride[p] = recon->stride[p];
        A.sstride[p] = src->stride[p];
    }
    A.width   = recon->width;
    A.height  = recon->height;
    A.b8_cols = s->geo.b8_cols;
    A.nhfb    = s->geo.nhfb;
    A.mask    = s->mask_all ? nullptr : s->d_mask;
    A.mse     = s->d_mse;
    A.skip    = s->d_skip;
    A.dir     = s->d_dir;
    A.var     = s->d_var;
    A.rem     = s->d_fb_kind ? s->d_mse_rem : nullptr;
    A.nfb     = s->nfb;
    A.fb0     = s->fb_rect[1] * s->geo.nhfb + s->fb_rect[0];
    A.fbw     = s->fb_rect[2] - s->fb_rect[0];
    A.cs      = recon->bit_depth - 8;
    A.ss      = subsampling;
    A.damping = damping;
    A.tab     = *tab;
    const dim3 grid((s->fb_rect[3] - s->fb_rect[1]) * A.fbw);
    A.wgclk = svtgpu_wgclk_begin((int)grid.x);
    if (recon->bit_depth > 8)
        hipLaunchKernelGGL(cdef_search_kernel<uint16_t>, grid, dim3(NT), 0, st, A);
    else
        hipLaunchKernelGGL(cdef_search_kernel<uint8_t>, grid, dim3(NT), 0, st, A);
    HIP_TRY(hipGetLastError());
    svtgpu_wgclk_end("cdef_search", (int)grid.x, st);
    return SVTGPU_OK;
}
