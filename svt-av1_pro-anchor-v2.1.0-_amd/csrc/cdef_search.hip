// cdef_search.hip — fused CDEF strength search for whole frames (SB64), gfx950.
//
// ≙ cdef_seg_search over all segments (Source/Lib/Encoder/Codec/EbCdefProcess.c:114-357):
// for every 64x64 filter block (FB), every plane and every candidate strength, filter the listed
// 8x8 (luma) / 4x4 (chroma) blocks (svt_cdef_filter_fb, EbCdef.c:339) and measure the distortion
// against the source (compute_cdef_dist, EbCdefProcess.c:87 → EbEncCdef.c:129/175).
//
// One workgroup (256 lanes, 4 waves) per FB.  The DLF output tile (+-2 px context, 0x7F7F outside
// the frame, exactly the samples the reference stages, EbCdefProcess.c:206-236) lives in LDS.
// Each lane owns two horizontally adjacent pixel PAIRS (4 px).  For a fixed direction the 12 tap
// differences |p - x| and their signs are strength-independent, so they are computed once per
// pass and kept in registers as packed int16 pairs; the strength loop is then pure packed-int16
// VALU (v_pk_lshrrev/sub/max/min/mad: 5 ops per tap pair) — no LDS traffic per strength.
// Per-8x8 luma statistics (sum d, sum d^2, sum (d-s)^2) reduce over the block's 16 lanes with DPP;
// the double-precision SSIM-like distortion (EbEncCdef.c:42-47) is evaluated once per
// (strength, block) in a lane-parallel epilogue.  Chroma SSE reduces through LDS atomics.
#include "cdef_common.h"

#define NT 256
#define LT 68 // luma tile: rows/cols -2..65
#define CT 36 // chroma tile: rows/cols -2..33

struct SearchArgs {
    const void *rec[3];
    const void *src[3];
    int32_t     rstride[3], sstride[3];
    int32_t     width, height;
    int32_t     b8_cols, nhfb;
    const uint8_t *mask;
    uint64_t   *mse;   // [2][nfb][64]
    uint8_t    *skip;  // [nfb]
    uint8_t    *dir;   // [nfb][64]
    int32_t    *var;   // [nfb][64]
    int32_t     nfb, fb0;
    int32_t     cs, ss, damping;
    CdefStrengthTable tab;
};

struct PxPair { // two horizontally adjacent samples, packed int16 (lo = left, hi = right)
    s16x2 x, lo, hi;
    s16x2 ad[12]; // |tap - x|: [0..1] pri k0 (+,-), [2..3] pri k1, [4..7] sec k0, [8..11] sec k1
    s16x2 sg[12]; // sign(tap - x) as +-1
};

template <typename T>
__device__ __forceinline__ uint16_t ld_px(const void *base, long idx) {
    return (uint16_t)((const T *)base)[idx];
}

// Stage a plane tile (rows r0-2 .. r0+n+1, cols c0-2 .. c0+n+1) into LDS, 0x7F7F outside the plane.
template <typename T>
__device__ void stage_tile(uint16_t *tile, int ts, int n, const void *plane, int stride, int pw, int ph, int r0,
                           int c0) {
    const int span = n + 2 * CDEF_BORDER;
    for (int i = threadIdx.x; i < span * span; i += NT) {
        const int r = i / span, c = i - r * span;
        const int fr = r0 + r - CDEF_BORDER, fc = c0 + c - CDEF_BORDER;
        uint16_t  v  = CDEF_VERY_LARGE_V;
        if (fr >= 0 && fc >= 0 && fr < ph && fc < pw)
            v = ld_px<T>(plane, (long)fr * stride + fc);
        tile[r * ts + c] = v;
    }
}

// Neighbourhood of the pair at tile position (r, c), (r, c+1) for direction `dir`.
__device__ __forceinline__ void load_pair(PxPair &P, const uint16_t *tile, int ts, int r, int c, int dir) {
    const uint16_t *p0 = tile + (r + CDEF_BORDER) * ts + (c + CDEF_BORDER);
    const int        xa = (int16_t)p0[0], xb = (int16_t)p0[1];
    int              loa = xa, hia = xa, lob = xb, hib = xb;
    const int        ds0 = (dir + 2) & 7, ds1 = (dir + 6) & 7;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int o[6] = {cdef_dir_dy(dir, k) * ts + cdef_dir_dx(dir, k), -(cdef_dir_dy(dir, k) * ts + cdef_dir_dx(dir, k)),
                          cdef_dir_dy(ds0, k) * ts + cdef_dir_dx(ds0, k), -(cdef_dir_dy(ds0, k) * ts + cdef_dir_dx(ds0, k)),
                          cdef_dir_dy(ds1, k) * ts + cdef_dir_dx(ds1, k), -(cdef_dir_dy(ds1, k) * ts + cdef_dir_dx(ds1, k))};
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const int va = (int16_t)p0[o[t]], vb = (int16_t)p0[o[t] + 1];
            if (va != CDEF_VERY_LARGE_V) hia = max(hia, va);
            if (vb != CDEF_VERY_LARGE_V) hib = max(hib, vb);
            loa = min(loa, va);
            lob = min(lob, vb);
            const int da = va - xa, db = vb - xb;
            // slot: pri taps (t<2) -> 2k + t ; sec taps -> 4 + 4k + (t-2)
            const int slot = t < 2 ? 2 * k + t : 4 + 4 * k + (t - 2);
            P.ad[slot] = (s16x2){(short)abs(da), (short)abs(db)};
            P.sg[slot] = (s16x2){(short)(da < 0 ? -1 : 1), (short)(db < 0 ? -1 : 1)};
        }
    }
    P.x  = (s16x2){(short)xa, (short)xb};
    P.lo = (s16x2){(short)loa, (short)lob};
    P.hi = (s16x2){(short)hia, (short)hib};
}

// Filter one pair with thresholds/shifts broadcast in both halves (EbCdef.c:253-300 in packed form:
// constrain(d) * tap == sign(d) * min(|d|, max(0, thr - (|d| >> shift))) * tap).
__device__ __forceinline__ s16x2 filter_pair(const PxPair &P, s16x2 pthr, u16x2 psh, s16x2 sthr, u16x2 ssh, short w0,
                                             short w1) {
    const s16x2 z = {0, 0};
    s16x2       acc[4] = {z, z, z, z};
#pragma unroll
    for (int t = 0; t < 12; t++) {
        const bool  pri = t < 4;
        const s16x2 thr = pri ? pthr : sthr;
        const u16x2 sh  = pri ? psh : ssh;
        const s16x2 a   = (s16x2)(((u16x2)P.ad[t]) >> sh);
        const s16x2 c   = __builtin_elementwise_max(thr - a, z);
        const s16x2 e   = __builtin_elementwise_min(P.ad[t], c);
        const int   cls = t < 2 ? 0 : t < 4 ? 1 : t < 8 ? 2 : 3;
        acc[cls]        = acc[cls] + e * P.sg[t];
    }
    const s16x2 sum = acc[0] * (s16x2){w0, w0} + acc[1] * (s16x2){w1, w1} + (acc[2] << (s16x2){1, 1}) + acc[3];
    const s16x2 rnd = (sum + (s16x2){8, 8} + (sum >> (s16x2){15, 15})) >> (s16x2){4, 4};
    const s16x2 y   = P.x + rnd;
    return __builtin_elementwise_max(__builtin_elementwise_min(y, P.hi), P.lo);
}

__device__ __forceinline__ s16x2 splat16(int v) { return (s16x2){(short)v, (short)v}; }
__device__ __forceinline__ u16x2 splatu16(int v) { return (u16x2){(unsigned short)v, (unsigned short)v}; }

template <typename T>
__global__ void __launch_bounds__(NT) cdef_search_kernel(const SearchArgs A) {
    __shared__ uint16_t ltile[LT * LT];
    __shared__ uint16_t ctile[2][CT * CT];
    __shared__ uint32_t stats[64][16][3];  // per pass: [gi][block-in-pass][sum_d, sum_d2, sse]
    __shared__ uint32_t sstat[64][2];      // per block source sum, sum^2 (luma)
    __shared__ uint64_t acc_l[64];         // per gi luma distortion
    __shared__ uint32_t acc_c[2][64];      // per gi chroma SSE per plane
    __shared__ int32_t  dcost[64][8];
    __shared__ uint8_t  sdir[64];
    __shared__ int32_t  svar[64];
    __shared__ uint8_t  slisted[64];
    __shared__ int32_t  nlisted;

    const int fb = A.fb0 + blockIdx.x;
    const int fbr = fb / A.nhfb, fbc = fb - fbr * A.nhfb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cs = A.cs;

    // ---- block list (svt_sb_compute_cdef_list, EbEncCdef.c:238-282) ----
    if (tid == 0) nlisted = 0;
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
            A.mse[(size_t)fb * 64 + tid]         = 0;
            A.mse[((size_t)A.nfb + fb) * 64 + tid] = 0;
            A.dir[(size_t)fb * 64 + tid]         = 0;
            A.var[(size_t)fb * 64 + tid]         = 0;
        }
        return;
    }

    // ---- stage tiles ----
    stage_tile<T>(ltile, LT, 64, A.rec[0], A.rstride[0], A.width, A.height, 64 * fbr, 64 * fbc);
    stage_tile<T>(ctile[0], CT, 32, A.rec[1], A.rstride[1], A.width >> 1, A.height >> 1, 32 * fbr, 32 * fbc);
    stage_tile<T>(ctile[1], CT, 32, A.rec[2], A.rstride[2], A.width >> 1, A.height >> 1, 32 * fbr, 32 * fbc);
    __syncthreads();

    // ---- direction per 8x8 luma block (svt_aom_cdef_find_dir_c, EbCdef.c:150-210) ----
    // wave w computes directions 2w and 2w+1 for block = lane (direction wave-uniform)
    {
        const int b = lane, by = b >> 3, bx = b & 7;
        int       xv[64];
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 8; j++)
                xv[i * 8 + j] = ((int)ltile[(8 * by + i + CDEF_BORDER) * LT + 8 * bx + j + CDEF_BORDER] >> cs) - 128;
        const int w840[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
#pragma unroll
        for (int dd = 0; dd < 2; dd++) {
            const int d = 2 * wave + dd;
            int       line[15];
#pragma unroll
            for (int k = 0; k < 15; k++) line[k] = 0;
            int cost = 0;
            switch (d) { // partial-sum line of sample (i, j) per direction (EbCdef.c:171-179)
#define ACC(EXPR)                                                                  \
    _Pragma("unroll") for (int i = 0; i < 8; i++) _Pragma("unroll") for (int j = 0; j < 8; j++) line[EXPR] += xv[i * 8 + j];
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
    const CdefStrengthTable &tab = A.tab;

    // ================= luma: 4 passes of 16 blocks =================
    for (int pass = 0; pass < 4; pass++) {
        const int bip = 4 * wave + (lane >> 4); // block in pass
        const int b = 16 * pass + bip, by = b >> 3, bx = b & 7;
        const int q = lane & 15, row = q >> 1, col0 = (q & 1) * 4;
        const int r = 8 * by + row, c = 8 * bx + col0;
        const bool listed = slisted[b];
        const bool valid = listed && (row % ss == 0);
        const uint32_t vmask = valid ? 0xFFFFFFFFu : 0u;
        // source samples (registers), zeroed outside the measured set
        s16x2 sp[2] = {{0, 0}, {0, 0}};
        if (valid) {
            const long o = (long)(64 * fbr + r) * A.sstride[0] + 64 * fbc + c;
            sp[0] = (s16x2){(short)ld_px<T>(A.src[0], o), (short)ld_px<T>(A.src[0], o + 1)};
            sp[1] = (s16x2){(short)ld_px<T>(A.src[0], o + 2), (short)ld_px<T>(A.src[0], o + 3)};
        }
        {
            uint32_t s1 = 0, s2 = 0;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                s1 = __builtin_amdgcn_udot2((u16x2)sp[h], (u16x2){1, 1}, s1, false);
                s2 = __builtin_amdgcn_udot2((u16x2)sp[h], (u16x2)sp[h], s2, false);
            }
            s1 = row16_sum(s1);
            s2 = row16_sum(s2);
            if (q == 0) {
                sstat[b][0] = s1;
                sstat[b][1] = s2;
            }
        }
        const int   vb = svar[b];
        const int   ib = (vb >> 6) ? min(msb32_dev((uint32_t)(vb >> 6)), 12) : 0;
        PxPair P[2];
        for (int grp = 0; grp < 2; grp++) {
            const int     n   = grp ? tab.n_luma_b : tab.n_luma_a;
            const int8_t *lst = grp ? tab.luma_b : tab.luma_a;
            if (n == 0) continue;
            const int d = grp ? sdir[b] : 0;
            load_pair(P[0], ltile, LT, r, c, d);
            load_pair(P[1], ltile, LT, r, c + 2, d);
            for (int k = 0; k < n; k++) {
                const int gi = lst[k];
                const int code = tab.code[gi];
                const int level = code >> 2;
                int       sec = code & 3;
                sec += sec == 3;
                const int pri  = level << cs;
                const int t    = vb ? (pri * (4 + ib) + 8) >> 4 : 0; // adjust_strength
                const int secs = sec << cs;
                const int psh  = max(0, ldamp - msb32_dev((uint32_t)t));
                const int ssh  = max(0, ldamp - msb32_dev((uint32_t)secs));
                const int odd  = (t >> cs) & 1;
                uint32_t sd = 0, sd2 = 0, sse = 0;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    s16x2 y = filter_pair(P[h], splat16(t), splatu16(psh), splat16(secs), splatu16(ssh),
                                          (short)(odd ? 3 : 4), (short)(odd ? 3 : 2));
                    y                = (s16x2)((u16x2)y & (u16x2){(unsigned short)vmask, (unsigned short)vmask});
                    const s16x2 diff = y - sp[h];
                    sd  = __builtin_amdgcn_udot2((u16x2)y, (u16x2){1, 1}, sd, false);
                    sd2 = __builtin_amdgcn_udot2((u16x2)y, (u16x2)y, sd2, false);
                    sse = (uint32_t)__builtin_amdgcn_sdot2(diff, diff, (int)sse, false);
                }
                sd  = row16_sum(sd);
                sd2 = row16_sum(sd2);
                sse = row16_sum(sse);
                if (q == 0) {
                    stats[gi][bip][0] = sd;
                    stats[gi][bip][1] = sd2;
                    stats[gi][bip][2] = sse;
                }
            }
        }
        __syncthreads();
        // double-precision distortion per (gi, block): 4 lanes per gi, 4 blocks per lane
        {
            const int gi = tid >> 2, sub = tid & 3;
            unsigned long long acc = 0;
            if (gi < tab.nstr) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int bb = 4 * sub + u, bg = 16 * pass + bb;
                    if (!slisted[bg]) continue;
                    acc += cdef_luma_dist(stats[gi][bb][0], sstat[bg][0], stats[gi][bb][1], sstat[bg][1],
                                          stats[gi][bb][2], cs);
                }
            }
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            if (sub == 0 && gi < tab.nstr) acc_l[gi] += acc;
        }
        __syncthreads();
    }

    // ================= chroma: one pass per plane =================
    for (int pl = 0; pl < 2; pl++) {
        const int cb = tid >> 2, by = cb >> 3, bx = cb & 7, row = tid & 3;
        const int r = 4 * by + row, c = 4 * bx;
        const bool valid = slisted[cb];
        s16x2 sp[2] = {{0, 0}, {0, 0}};
        if (valid) {
            const long o = (long)(32 * fbr + r) * A.sstride[1 + pl] + 32 * fbc + c;
            sp[0] = (s16x2){(short)ld_px<T>(A.src[1 + pl], o), (short)ld_px<T>(A.src[1 + pl], o + 1)};
            sp[1] = (s16x2){(short)ld_px<T>(A.src[1 + pl], o + 2), (short)ld_px<T>(A.src[1 + pl], o + 3)};
        }
        const uint32_t vmask = valid ? 0xFFFFFFFFu : 0u;
        PxPair P[2];
        for (int grp = 0; grp < 2; grp++) {
            const int     n   = grp ? tab.n_chroma_b : tab.n_chroma_a;
            const int8_t *lst = grp ? tab.chroma_b : tab.chroma_a;
            if (n == 0) continue;
            const int d = grp ? sdir[cb] : 0;
            load_pair(P[0], ctile[pl], CT, r, c, d);
            load_pair(P[1], ctile[pl], CT, r, c + 2, d);
            for (int k = 0; k < n; k++) {
                const int gi = lst[k];
                const int code = tab.code[gi];
                int       sec = code & 3;
                sec += sec == 3;
                const int pri  = (code >> 2) << cs;
                const int secs = sec << cs;
                const int psh  = max(0, cdamp - msb32_dev((uint32_t)pri));
                const int ssh  = max(0, cdamp - msb32_dev((uint32_t)secs));
                const int odd  = (pri >> cs) & 1;
                uint32_t sse = 0;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    s16x2 y = filter_pair(P[h], splat16(pri), splatu16(psh), splat16(secs), splatu16(ssh),
                                          (short)(odd ? 3 : 4), (short)(odd ? 3 : 2));
                    y                = (s16x2)((u16x2)y & (u16x2){(unsigned short)vmask, (unsigned short)vmask});
                    const s16x2 diff = y - sp[h];
                    sse = (uint32_t)__builtin_amdgcn_sdot2(diff, diff, (int)sse, false);
                }
                sse = row16_sum(sse);
                if ((lane & 15) == 0) atomicAdd(&acc_c[pl][gi], sse);
            }
        }
    }
    __syncthreads();

    // ---- per-FB mse rows (EbCdefProcess.c:293-298, :349-353) ----
    if (tid < 64) {
        const int gi = tid;
        uint64_t  m0 = 0, m1 = 0;
        if (gi < tab.nstr) {
            m0 = (acc_l[gi] >> (2 * cs)) * (uint64_t)ss;
            m1 = tab.uv_on[gi] ? ((uint64_t)(acc_c[0][gi] >> (2 * cs)) + (uint64_t)(acc_c[1][gi] >> (2 * cs)))
                               : 1040400ull * 64; // default_mse_uv * 64
        }
        A.mse[(size_t)fb * 64 + gi]             = m0;
        A.mse[((size_t)A.nfb + fb) * 64 + gi]   = m1;
        if (tid == 0) A.skip[fb] = 0;
    }
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
    A.nfb     = s->nfb;
    A.fb0     = s->fb_row_begin * s->geo.nhfb;
    A.cs      = recon->bit_depth - 8;
    A.ss      = subsampling;
    A.damping = damping;
    A.tab     = *tab;
    if (recon->bit_depth > 8)
        hipLaunchKernelGGL(cdef_search_kernel<uint16_t>, dim3((s->fb_row_end - s->fb_row_begin) * s->geo.nhfb), dim3(NT), 0, st, A);
    else
        hipLaunchKernelGGL(cdef_search_kernel<uint8_t>, dim3((s->fb_row_end - s->fb_row_begin) * s->geo.nhfb), dim3(NT), 0, st, A);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}
