// ccso.hip — CCSO, the fork's cross-component sample offset, on the MI355X.
//
// The reference (EbPickccso.c:464-779, derive_ccso_filter) trains 200 configurations per plane -- band-offset-only or
// not x 6 filter supports x 4 quantization steps x 2 edge classifiers x 1-128 bands -- and each training pass filters a
// copy of the whole plane and measures every filter block's SSD.  Here the plane is read ONCE per filter support:
//
//   ccso_bins_kernel     per filter block and filter support, a histogram over (fine band, bucket of the first
//                        neighbour difference, bucket of the second): count, sum of (org - rec), sum of its square, and
//                        for the samples a table offset can clamp (rec < 10 or rec > max - 7) the exact correction of
//                        the squared error per table offset.  The 9 buckets split the differences at every threshold
//                        any quantization step uses (+-8/16/32/64), so every (step, classifier) class is a union of
//                        buckets.  One pass more for the band-offset-only bins (128 fine bands).
//   ccso_merge_kernel    per (support, step, classifier) combination and block: the fine classes (8 bands x 3 x 3) with
//                        count, error sum and the block SSD under each of the 8 possible table offsets
//                        (S2 - 2 o S1 + o^2 n + clamp correction: exact integers).
//   ccso_train_kernel    one wave per configuration runs the reference's training loop on those moments: the class
//                        errors of the enabled blocks -> the table (derive_lut_offset, the reference's float
//                        arithmetic) -> each block's filtered SSD as a sum of table-indexed moments -> the block
//                        decisions (derive_blk_md) -> the RD cost (count_lut_bits, RDCOST_DBL) -> stop rule.
//   ccso_final_kernel    the reference's loop-order choice over the configurations and the unfiltered comparison;
//                        writes the plane's SvtGpuCcsoParams and block flags in device memory.
//   ccso_apply_kernel    ccso_frame's per-plane filter (EbCcso.c:297-677), in place, 8- or 16-bit planes.
//
// Every number is an integer or the reference's own float/double expression, so the result is bit-exact (pinned by
// tests/golden/ccso.bin through oracle/ccso_oracle.c).  Roofline: the bins pass is HBM-bound -- per sample 2 B org +
// 2 B rec + the luma centre and its two neighbours (L2 hits after the first support) -- 7 passes over the plane.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "svtgpu_internal.h"

namespace {
constexpr int PAD     = SVTGPU_CCSO_PAD;
constexpr int NSUP    = 6;            // filter supports (derive_ccso_sample_pos, EbCcso.c:204-234)
constexpr int NKIND   = NSUP + 1;     // + band-offset-only
constexpr int NBIN    = 8 * 9 * 9;    // fine band x bucket x bucket
constexpr int NFINE   = 128;          // fine classes per merged moment slot (72 used by the edge combinations)
constexpr int NCOMBO  = NSUP * 4 * 2; // support x quantization step x edge classifier
constexpr int NCFG    = NCOMBO * 4 + 8;
constexpr int MAXNB   = 1024;         // filter blocks per plane (an 8192 x 8192 picture has 32 x 32)
constexpr int STRIP   = 64;           // most rows of a block per bins workgroup (Planes::strip: 32 or 64)
constexpr int BTHREADS = 256;

__constant__ int kOff[8] = {-10, -7, -3, -1, 0, 1, 3, 7}; // ccso_offset (EbPickccso.c:43)

struct Bin {            // one histogram cell (global); corr[o] = sum of clamped - unclamped squared errors
    uint32_t n, s1;
    uint64_t s2;
    uint64_t corr[8];
};
// The moments of one (plane, combination): 9 arrays of nbp x NFINE words (block-major, fine class minor) -- count << 32
// | error sum, then the block SSD under each of the 8 table offsets.  Structure of arrays: a wave's loads of one field
// are contiguous.
constexpr int MOM_WORDS = 9;
__device__ __forceinline__ size_t mom_ssd(int k, size_t n) { return (size_t)(k + 1) * n; }
struct Geo {
    int32_t w, h, pw, ph, ss, log2, bs, nvfb, nhfb, nb, nbx, nby, nbp;
};

Geo geo_of(int w, int h, int plane) {
    Geo g;
    g.w = w, g.h = h, g.ss = plane > 0, g.pw = plane ? w >> 1 : w, g.ph = plane ? h >> 1 : h;
    g.log2 = plane ? 7 : 8, g.bs = 1 << g.log2;
    const int unit = g.bs >> 2, mi_rows = ((h + 7) & ~7) >> 2, mi_cols = ((w + 7) & ~7) >> 2;
    g.nvfb = ((mi_rows >> g.ss) + unit - 1) / unit, g.nhfb = ((mi_cols >> g.ss) + unit - 1) / unit;
    g.nb  = g.nvfb * g.nhfb;
    g.nbx = (g.pw + g.bs - 1) / g.bs, g.nby = (g.ph + g.bs - 1) / g.bs, g.nbp = g.nbx * g.nby;
    return g;
}

__host__ __device__ inline void sample_pos(int *loc, int stride, int sup) {
    switch (sup) {
    case 0: loc[0] = -stride, loc[1] = stride; break;
    case 1: loc[0] = -stride - 1, loc[1] = stride + 1; break;
    case 2: loc[0] = -1, loc[1] = 1; break;
    case 3: loc[0] = stride - 1, loc[1] = -stride + 1; break;
    case 4: loc[0] = -3, loc[1] = 3; break;
    default: loc[0] = -5, loc[1] = 5; break;
    }
}

// bucket of a neighbour difference: 0 d<-64 | 1 d<-32 | 2 d<-16 | 3 d<-8 | 4 |d|<=8 | 5 d<=16 | 6 d<=32 | 7 d<=64 | 8
__device__ __forceinline__ int bucket(int d) {
    return (d >= -64) + (d >= -32) + (d >= -16) + (d >= -8) + (d > 8) + (d > 16) + (d > 32) + (d > 64);
}
// class of a bucket under quantization step level L (8:1 16:2 32:3 64:4), cal_filter_support (EbCcso.c:238-259)
__device__ __forceinline__ int bucket_class(int b, int L, int clf) {
    if (b <= 4 - L) return 0;
    return (clf == 0 && b >= 4 + L) ? 2 : 1;
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

// ---------------------------------------------------------------------------------------------
// pass 1: histograms (grid: nbp * strips, NKIND)
// ---------------------------------------------------------------------------------------------
struct Planes { // the planes of one search launch: plane = plane0 + blockIdx.z (final: + blockIdx.x)
    Geo               g[3];
    const uint16_t   *ext, *org[3], *rec[3];
    Bin              *bins[3];  // [NKIND][nbp][NBIN]
    uint64_t         *mom[3];   // [NCOMBO + 1][MOM_WORDS][nbp][NFINE]
    double           *cost[3];  // [NCFG]
    int8_t           *lut[3];   // [NCFG][NFINE] offset of each merged class
    uint8_t          *ctrl[3];  // [NCFG][nb]
    SvtGpuCcsoParams *params[3];
    uint8_t          *flags[3];
    int32_t           bd, rdmult, plane0;
    int32_t           strip; // rows per bins workgroup: 64 for pictures of many blocks (fewer, longer workgroups), else 32
};

// LDS cells: the count and the squared-error sum share one 64-bit word (count << 50 | sum of squares: a workgroup sees
// at most 64 x 256 samples and 12-bit errors, so neither field overflows) and the error sum is kept biased by +4096 per
// sample (non-negative, < 2^26); every sample costs at most two LDS atomics, fewer where lanes share a bin
constexpr int      NQ_SHIFT = 49;
constexpr uint32_t S1_BIAS  = 4096;
constexpr int      RUN      = 4; // wave-wide bin groups summed per step before the per-lane atomics
constexpr int      U        = 8; // steps whose samples are loaded together

__global__ __launch_bounds__(BTHREADS) void ccso_bins_kernel(Planes a) {
    __shared__ unsigned long long s_nq[NBIN];
    __shared__ uint32_t           s_s1[NBIN];
    __shared__ int32_t            s_corr[8][NBIN]; // |clamped - unclamped| <= 10 * 2 * 4105 per sample: int32 per tile
    const int  tid = threadIdx.x, kind = blockIdx.y, pl = a.plane0 + blockIdx.z;
    const Geo &g = a.g[pl];
    const int  strips = g.bs / a.strip;
    if ((int)blockIdx.x >= g.nbp * strips) return;
    const int  pb = blockIdx.x / strips, strip = blockIdx.x % strips;
    const uint16_t *org = a.org[pl], *rec = a.rec[pl];
    const int  bx = pb % g.nbx, by = pb / g.nbx;
    const int  x0 = bx * g.bs, y0 = by * g.bs + strip * a.strip;
    const int  nbins = kind < NSUP ? NBIN : 128;
    for (int i = tid; i < nbins; i += BTHREADS) {
        s_nq[i] = 0, s_s1[i] = 0;
        for (int o = 0; o < 8; o++) s_corr[o][i] = 0;
    }
    __syncthreads();
    const int rows = min(a.strip, min(g.bs - strip * a.strip, g.ph - y0)), cols = min(g.bs, g.pw - x0);
    if (rows > 0 && cols > 0) {
        const int es = g.w + 2 * PAD, maxv = (1 << a.bd) - 1;
        int       loc[2];
        sample_pos(loc, es, kind < NSUP ? kind : 0);
        const int sh = kind < NSUP ? a.bd - 3 : a.bd - 7;
        // lane-contiguous columns (coalesced loads of org / rec / the luma row), rps rows per step; the samples of U
        // steps are loaded before any is binned, so a wave keeps 5 U loads in flight instead of waiting on each row
        const int rps = BTHREADS / cols, col = tid % cols, row0 = tid / cols, xx = x0 + col;
        const bool nb2 = kind < NSUP;
        for (int rb = 0; rb < rows; rb += rps * U) { // uniform trip count: the flushes below are convergent
            int vc[U], v0[U], v1[U], vo[U], vr[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int ry = rb + row0 + u * rps;
                vc[u] = -1;
                if (row0 < rps && ry < rows) {
                    const int       yy = y0 + ry;
                    const uint16_t *c  = a.ext + (size_t)(PAD + (yy << g.ss)) * es + PAD + (xx << g.ss);
                    vc[u] = c[0], vo[u] = org[(size_t)yy * g.w + xx], vr[u] = rec[(size_t)yy * g.w + xx];
                    if (nb2) v0[u] = c[loc[0]], v1[u] = c[loc[1]];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                int                cur = -1;
                unsigned long long nq  = 0;
                uint32_t           s1  = 0;
                if (vc[u] >= 0) {
                    const int cv = vc[u], o = vo[u], r = vr[u], e = o - r;
                    cur = cv >> sh;
                    if (nb2) cur = (cur * 9 + bucket(v0[u] - cv)) * 9 + bucket(v1[u] - cv);
                    nq = (1ull << NQ_SHIFT) + (unsigned long long)(e * e);
                    s1 = (uint32_t)(e + (int)S1_BIAS);
                    if (r < 10 || r > maxv - 7)
                        for (int k = 0; k < 8; k++) {
                            const int f = clampi(r + kOff[k], 0, maxv), d = o - f, w = e - kOff[k];
                            if (d * d != w * w) atomicAdd(&s_corr[k][cur], d * d - w * w);
                        }
                }
                // lanes in one bin are summed across the wave first (smooth content puts most of a wave in a few
                // bins: one LDS atomic per bin instead of one per lane); small groups add directly
                unsigned long long rem = __ballot(cur >= 0);
                for (int t = 0; t < RUN && rem; t++) {
                    const int                b    = __builtin_amdgcn_readlane(cur, __ffsll((long long)rem) - 1);
                    const bool               mine = cur == b;
                    const unsigned long long m    = __ballot(mine);
                    if (__popcll(m) < 4) break;
                    const unsigned long long v = wave_sum_lane63(mine ? nq : 0ull);
                    const uint32_t           w = wave_sum_u32_lane63(mine ? s1 : 0u);
                    if ((tid & 63) == 63) atomicAdd(&s_nq[b], v), atomicAdd(&s_s1[b], w);
                    if (mine) cur = -1;
                    rem &= ~m;
                }
                if (cur >= 0) atomicAdd(&s_nq[cur], nq), atomicAdd(&s_s1[cur], s1);
            }
        }
    }
    __syncthreads();
    Bin *out = a.bins[pl] + ((size_t)kind * g.nbp + pb) * NBIN;
    for (int i = tid; i < nbins; i += BTHREADS) {
        const unsigned long long nq = s_nq[i];
        const uint32_t           n  = (uint32_t)(nq >> NQ_SHIFT);
        if (!n) continue;
        atomicAdd(&out[i].n, n);
        atomicAdd(&out[i].s1, s_s1[i] - S1_BIAS * n);
        atomicAdd((unsigned long long *)&out[i].s2, nq & ((1ull << NQ_SHIFT) - 1));
        for (int k = 0; k < 8; k++)
            if (s_corr[k][i]) atomicAdd((unsigned long long *)&out[i].corr[k], (unsigned long long)(long long)s_corr[k][i]);
    }
}

// ---------------------------------------------------------------------------------------------
// pass 2: moments per combination (grid: nbp, NKIND; the support's 648 bins of one block staged in LDS once, its 8
// (quantization step, classifier) combinations x 72 fine classes summed from there)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ccso_merge_kernel(Planes a) {
    __shared__ Bin s_bin[NBIN];
    const int tid = threadIdx.x, pb = blockIdx.x, kind = blockIdx.y, pl = a.plane0 + blockIdx.z, nbp = a.g[pl].nbp;
    if (pb >= nbp) return;
    const Bin *bins = a.bins[pl];
    uint64_t  *mom  = a.mom[pl];
    const size_t N  = (size_t)nbp * NFINE;
    const int  nbins = kind < NSUP ? NBIN : 128;
    const Bin *src   = bins + ((size_t)kind * nbp + pb) * NBIN;
    {
        const uint64_t *s = (const uint64_t *)src;
        uint64_t       *d = (uint64_t *)s_bin;
#pragma unroll 8
        for (int i = tid; i < nbins * (int)(sizeof(Bin) / 8); i += 256) d[i] = s[i];
    }
    __syncthreads();
    constexpr int BW = (int)(sizeof(Bin) / 8); // words per cell: count | error sum (two u32), square sum, 8 corrections
    if (kind < NSUP) { // running sums along the second bucket (every class is a range of buckets): in place, per word
        for (int t = tid; t < 72 * BW; t += 256) {
            const int row = t / BW, w = t % BW;
            uint64_t *c   = (uint64_t *)(s_bin + row * 9) + w;
            if (w == 0) { // the two u32 fields (n low, s1 high) add separately (the error sum wraps)
                uint32_t an = 0, as = 0;
                for (int j = 0; j < 9; j++) {
                    an += (uint32_t)c[j * BW], as += (uint32_t)(c[j * BW] >> 32);
                    c[j * BW] = (uint64_t)as << 32 | an;
                }
            } else {
                uint64_t acc = 0;
                for (int j = 0; j < 9; j++) acc += c[j * BW], c[j * BW] = acc;
            }
        }
        __syncthreads();
    }
    const int nout = kind < NSUP ? 8 * 72 : 128;
    for (int o = tid; o < nout; o += 256) {
        uint32_t n = 0, s1 = 0;
        uint64_t s2 = 0, corr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int      combo, f;
        if (kind < NSUP) {
            const int qc = o / 72, qi = qc >> 1, clf = qc & 1;
            const int L  = qi == 0 ? 2 : qi == 1 ? 1 : qi == 2 ? 3 : 4; // quant_sz {16, 8, 32, 64}
            f = o % 72, combo = (kind * 4 + qi) * 2 + clf;
            const int band = f / 9, c0 = (f / 3) % 3, c1 = f % 3;
            // the bucket range of a class (bucket_class): 0 [0, 4 - L]; 1 [5 - L, 3 + L] (clf 0) or [5 - L, 8];
            // 2 [4 + L, 8] (clf 0 only)
            auto lo = [&](int c) { return c == 0 ? 0 : c == 1 ? 5 - L : 4 + L; };
            auto hi = [&](int c) { return c == 0 ? 4 - L : c == 1 ? (clf ? 8 : 3 + L) : (clf ? -1 : 8); };
            const int l1 = lo(c1), h1 = hi(c1);
            if (h1 >= l1)
                for (int b0 = lo(c0); b0 <= hi(c0); b0++) {
                    const uint64_t *r = (const uint64_t *)(s_bin + band * 81 + b0 * 9);
                    const uint64_t *u = r + h1 * BW, *v = l1 ? r + (l1 - 1) * BW : nullptr;
                    n += (uint32_t)u[0] - (v ? (uint32_t)v[0] : 0u);
                    s1 += (uint32_t)(u[0] >> 32) - (v ? (uint32_t)(v[0] >> 32) : 0u);
                    s2 += u[1] - (v ? v[1] : 0ull);
                    for (int k = 0; k < 8; k++) corr[k] += u[2 + k] - (v ? v[2 + k] : 0ull);
                }
        } else {
            f = o, combo = NCOMBO;
            const Bin &x = s_bin[f];
            n = x.n, s1 = x.s1, s2 = x.s2;
            for (int k = 0; k < 8; k++) corr[k] = x.corr[k];
        }
        uint64_t     *m  = mom + (size_t)combo * MOM_WORDS * N + (size_t)pb * NFINE + f;
        const int64_t S1 = (int32_t)s1;
        m[0]             = (uint64_t)n << 32 | s1;
        for (int k = 0; k < 8; k++)
            m[mom_ssd(k, N)] = s2 - (uint64_t)(2 * kOff[k] * S1) + (uint64_t)(kOff[k] * kOff[k]) * n + corr[k];
    }
}

// ---------------------------------------------------------------------------------------------
// pass 3: the training loop of every configuration (grid NCFG; one wave each)
// ---------------------------------------------------------------------------------------------

// RDCOST_DBL_WITH_NATIVE_BD_DIST1 (EbPickccso.h:9) over RDCOST_DBL (EbRestoration.h:346); -ffp-contract=off
__device__ __host__ inline double rdcost(int rdmult, int bits, uint64_t dist, int bd) {
    const double d = (double)(dist >> (2 * (bd - 8)));
    return (((double)bits * rdmult) / (double)(1 << 9)) + (d * (1 << 7));
}

// derive_lut_offset for one class (EbPickccso.c:439-456): the index of the chosen offset in kOff.  The reference's
// float quotient is the correctly rounded one; the double quotient of the two float operands rounded to float is it.
__device__ int lut_offset_index(int32_t err, int32_t cnt) {
    if (!cnt) return 4;
    const float t = (float)((double)(float)err / (double)(float)cnt);
    if (t < -10.0f) return 0;
    if (t >= 7.0f) return 7;
    for (int k = 0; k < 7; k++)
        if (t >= (float)kOff[k] && t <= (float)kOff[k + 1]) {
            const float lo = t - (float)kOff[k], hi = t - (float)kOff[k + 1];
            return fabsf(lo) > fabsf(hi) ? k + 1 : k;
        }
    return 4; // unreachable: [-10, 7) is covered
}
// count_lut_bits of one class (EbPickccso.c:360-378): the position in {0, 1, -1, 3, -3, 7, -7, -10}, capped at 7
__device__ __forceinline__ int lut_bits_of(int k) {
    constexpr int pos[8] = {7, 7, 5, 3, 1, 2, 4, 6}; // kOff index -> 1 + index in the reordered list (capped)
    return pos[k];
}

constexpr int TT = 512; // threads per configuration: the moment loads of a training pass spread over 8 waves
constexpr int LU = 4;   // moments loaded per thread before they are accumulated

__global__ __launch_bounds__(TT) void ccso_train_kernel(Planes a) {
    __shared__ uint8_t            s_ctrl[MAXNB], s_best[MAXNB];
    __shared__ unsigned long long s_unf[MAXNB], s_trn[MAXNB];
    __shared__ uint32_t           s_err[NFINE], s_cnt[NFINE];
    __shared__ uint8_t            s_off[NFINE], s_boff[NFINE];
    __shared__ unsigned long long s_dist;
    __shared__ int                s_any, s_bits;
    const int  tid = threadIdx.x, cfg = blockIdx.x, pl = a.plane0 + blockIdx.z;
    const Geo &g   = a.g[pl];
    const int  bo = cfg >= NCOMBO * 4, k = bo ? cfg - NCOMBO * 4 : cfg & 3, combo = bo ? NCOMBO : cfg >> 2;
    const int  clf = bo ? 0 : combo & 1, edges = bo ? 1 : (clf ? 2 : 3), F = bo ? 128 : 72;
    const int  nb = g.nb, nbp = g.nbp, nbands = 1 << k;
    const size_t    N   = (size_t)nbp * NFINE;
    const uint64_t *mom = a.mom[pl] + (size_t)combo * MOM_WORDS * N;
    // the merged class of a fine class at this band count
    auto merged = [&](int f) { return bo ? f >> (7 - k) : ((f / 9) >> (3 - k)) * 9 + f % 9; };
    auto blk2d  = [&](int p) { return (p / g.nbx) * g.nhfb + p % g.nbx; };
    for (int i = tid; i < nb; i += TT) s_unf[i] = 0, s_ctrl[i] = 1, s_best[i] = 0;
    if (tid < NFINE) s_boff[tid] = 4;
    __syncthreads();
    for (int i0 = tid; i0 < nbp * F; i0 += TT * LU) { // compute_distortion of the unfiltered plane
        unsigned long long v[LU];
#pragma unroll
        for (int u = 0; u < LU; u++) {
            const int i = i0 + u * TT;
            v[u]        = i < nbp * F ? mom[mom_ssd(4, N) + (size_t)(i / F) * NFINE + i % F] : 0;
        }
#pragma unroll
        for (int u = 0; u < LU; u++)
            if (v[u]) atomicAdd(&s_unf[blk2d((i0 + u * TT) / F)], v[u]);
    }
    __syncthreads();
    double best = DBL_MAX, prev = DBL_MAX;
    int    enable = 1;
    for (int iter = 0;; iter++) {
        int improvement = 0;
        if (enable) { // ccso_compute_class_err + derive_lut_offset
            if (tid < NFINE) s_err[tid] = 0, s_cnt[tid] = 0;
            __syncthreads();
            // the class errors of block p pair with the flag of index p (:211-233); LU moments loaded per round
            for (int i0 = tid; i0 < nbp * F; i0 += TT * LU) {
                uint32_t n[LU], e[LU];
#pragma unroll
                for (int u = 0; u < LU; u++) {
                    const int i = i0 + u * TT;
                    n[u]        = 0;
                    if (i < nbp * F && s_ctrl[i / F]) {
                        const uint64_t m = mom[(size_t)(i / F) * NFINE + i % F];
                        n[u] = (uint32_t)(m >> 32), e[u] = (uint32_t)m;
                    }
                }
#pragma unroll
                for (int u = 0; u < LU; u++)
                    if (n[u]) {
                        const int c = merged((i0 + u * TT) % F);
                        atomicAdd(&s_err[c], e[u]), atomicAdd(&s_cnt[c], n[u]);
                    }
            }
            __syncthreads();
            if (tid < NFINE) s_off[tid] = (uint8_t)lut_offset_index((int32_t)s_err[tid], (int32_t)s_cnt[tid]);
        }
        for (int i = tid; i < nb; i += TT) s_trn[i] = 0;
        if (tid == 0) s_dist = 0, s_any = 0, s_bits = 0;
        __syncthreads();
        for (int i0 = tid; i0 < nbp * F; i0 += TT * LU) { // the filtered plane's block SSDs
            unsigned long long v[LU];
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * TT;
                v[u] = i < nbp * F ? mom[mom_ssd(s_off[merged(i % F)], N) + (size_t)(i / F) * NFINE + i % F] : 0;
            }
#pragma unroll
            for (int u = 0; u < LU; u++)
                if (v[u]) atomicAdd(&s_trn[blk2d((i0 + u * TT) / F)], v[u]);
        }
        __syncthreads();
        if (enable) { // derive_blk_md: the rate it sums is never read (EbPickccso.c:666-687)
            unsigned long long d = 0;
            int                any = 0;
            for (int i = tid; i < nb; i += TT) {
                const int on = s_trn[i] < s_unf[i];
                s_ctrl[i]    = (uint8_t)on;
                d += on ? s_trn[i] : s_unf[i];
                any |= on;
            }
            if (d) atomicAdd(&s_dist, d);
            if (any) atomicOr(&s_any, 1);
            if (tid < NFINE) {
                const int c = tid, band = bo ? c : c / 9, d0 = bo ? 0 : (c / 3) % 3, d1 = bo ? 0 : c % 3;
                if (band < nbands && d0 < edges && d1 < edges) atomicAdd(&s_bits, lut_bits_of(s_off[c]));
            }
        }
        __syncthreads();
        enable = enable && s_any;
        if (enable) {
            const int    total = s_bits + (bo ? 5 : 10) + nb; // frame bits, EbPickccso.c:530-542 (CONFIG_CCSO_SIGFIX)
            const double cost  = rdcost(a.rdmult, total, s_dist, a.bd);
            if (cost < prev) prev = cost, improvement = 1;
            if (cost < best) {
                best = cost;
                if (tid < NFINE) s_boff[tid] = s_off[tid];
                for (int i = tid; i < nb; i += TT) s_best[i] = s_ctrl[i];
            }
        }
        __syncthreads();
        if (!improvement || iter + 1 > 15) break; // CCSO_MAX_ITERATIONS (EbPickccso.h:7)
    }
    if (tid == 0) a.cost[pl][cfg] = best;
    if (tid < NFINE) a.lut[pl][(size_t)cfg * NFINE + tid] = (int8_t)kOff[s_boff[tid]];
    for (int i = tid; i < nb; i += TT) a.ctrl[pl][(size_t)cfg * nb + i] = s_best[i];
}

// ---------------------------------------------------------------------------------------------
// pass 4: the plane's choice (one workgroup)
// ---------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void ccso_final_kernel(Planes a) {
    __shared__ int                s_win;
    __shared__ unsigned long long s_unf;
    __shared__ double             s_c[256];
    __shared__ int                s_i[256];
    const int         lane = threadIdx.x, pl = a.plane0 + blockIdx.x, nb = a.g[pl].nb;
    const uint64_t   *mom  = a.mom[pl];
    const size_t      N    = (size_t)a.g[pl].nbp * NFINE;
    const double     *cost = a.cost[pl];
    SvtGpuCcsoParams *prm  = a.params[pl];
    uint8_t          *flg  = a.flags[pl];
    if (lane == 0) s_unf = 0;
    __syncthreads();
    unsigned long long u = 0;
    for (int i = lane; i < a.g[pl].nbp * 72; i += 256) u += mom[mom_ssd(4, N) + (size_t)(i / 72) * NFINE + i % 72];
    atomicAdd(&s_unf, u);
    // the reference's loop order (EbPickccso.c:550-578) keeps the first strict minimum: the smallest cost, earliest
    // configuration among equals
    double c_min = DBL_MAX;
    int    i_min = -1;
    for (int c = lane; c < NCFG; c += 256)
        if (cost[c] < c_min) c_min = cost[c], i_min = c;
    s_c[lane] = c_min, s_i[lane] = i_min;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (lane < w) {
            const double c2 = s_c[lane + w];
            const int    i2 = s_i[lane + w];
            if (i2 >= 0 && (s_i[lane] < 0 || c2 < s_c[lane] || (c2 == s_c[lane] && i2 < s_i[lane])))
                s_c[lane] = c2, s_i[lane] = i2;
        }
        __syncthreads();
    }
    if (lane == 0) s_win = (s_i[0] >= 0 && !(rdcost(a.rdmult, 1, s_unf, a.bd) < s_c[0])) ? s_i[0] : -1;
    __syncthreads();
    const int win = s_win;
    uint8_t  *P   = (uint8_t *)prm;
    for (int i = lane; i < (int)sizeof(SvtGpuCcsoParams); i += 256) P[i] = 0;
    __syncthreads();
    if (win < 0) {
        for (int i = lane; i < nb; i += 256) flg[i] = 0;
        return;
    }
    const int bo = win >= NCOMBO * 4, k = bo ? win - NCOMBO * 4 : win & 3, combo = win >> 2;
    if (lane == 0) {
        prm->enable = 1, prm->bo_only = (uint8_t)bo, prm->max_band_log2 = (uint8_t)k;
        prm->quant_idx          = (uint8_t)(bo ? 0 : (combo >> 1) & 3);
        prm->ext_filter_support = (uint8_t)(bo ? 0 : combo >> 3);
        prm->edge_clf           = (uint8_t)(bo ? 0 : combo & 1);
    }
    const int edges = bo ? 1 : ((combo & 1) ? 2 : 3);
    for (int c = lane; c < NFINE; c += 256) {
        const int band = bo ? c : c / 9, d0 = bo ? 0 : (c / 3) % 3, d1 = bo ? 0 : c % 3;
        if (band < (1 << k) && d0 < edges && d1 < edges)
            prm->filter_offset[(band << 4) + (d0 << 2) + d1] = a.lut[pl][(size_t)win * NFINE + c];
    }
    for (int i = lane; i < nb; i += 256) flg[i] = a.ctrl[pl][(size_t)win * nb + i];
}

// ---------------------------------------------------------------------------------------------
// apply (ccso_frame's per-plane body) and the padded luma
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void ccso_apply_kernel(const uint16_t *ext, T *dst, int dst_stride,
                                                         const SvtGpuCcsoParams *prm, const uint8_t *flags, Geo g,
                                                         int bd) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= g.pw || y >= g.ph || !prm->enable) return;
    if (!flags[(y >> g.log2) * g.nhfb + (x >> g.log2)]) return;
    const int       es = g.w + 2 * PAD, maxv = (1 << bd) - 1;
    const uint16_t *c  = ext + (size_t)(PAD + (y << g.ss)) * es + PAD + (x << g.ss);
    int             c0 = 0, c1 = 0;
    if (!prm->bo_only) {
        int loc[2];
        sample_pos(loc, es, prm->ext_filter_support);
        const int q = prm->quant_idx == 0 ? 16 : prm->quant_idx == 1 ? 8 : prm->quant_idx == 2 ? 32 : 64;
        const int d0 = c[loc[0]] - c[0], d1 = c[loc[1]] - c[0];
        if (prm->edge_clf == 0) c0 = d0 > q ? 2 : d0 < -q ? 0 : 1, c1 = d1 > q ? 2 : d1 < -q ? 0 : 1;
        else c0 = d0 < -q ? 0 : 1, c1 = d1 < -q ? 0 : 1;
    }
    const int band = prm->max_band_log2 ? c[0] >> (bd - prm->max_band_log2) : 0;
    T        *d    = dst + (size_t)y * dst_stride + x;
    *d             = (T)clampi(prm->filter_offset[(band << 4) + (c0 << 2) + c1] + (int)*d, 0, maxv);
}

// one wave per padded row segment of 512 samples (8 per lane, lane-contiguous)
template <typename T>
__global__ __launch_bounds__(256) void ccso_extend_kernel(const T *luma, int stride, int w, int h, uint16_t *ext) {
    const int es = w + 2 * PAD, y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (y >= h + 2 * PAD) return;
    const T  *src = luma + (size_t)clampi(y - PAD, 0, h - 1) * stride;
    uint16_t *dst = ext + (size_t)y * es;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int x = blockIdx.x * 512 + k * 64 + (threadIdx.x & 63);
        if (x < es) dst[x] = src[clampi(x - PAD, 0, w - 1)];
    }
}

} // namespace

struct SvtGpuCcsoState {
    SvtGpuContext    *ctx;
    int32_t           width, height, nbp_max, nb_max;
    Bin              *bins; // per plane: [3][NKIND][nbp_max][NBIN] (the three planes' searches run in one launch)
    uint64_t         *mom;  // [3][NCOMBO + 1][MOM_WORDS][nbp_max][NFINE] (a plane's combinations use its own nbp)
    double           *cost; // [3][NCFG]
    int8_t           *lut;  // [3][NCFG][NFINE]
    uint8_t          *ctrl; // [3][NCFG][nb_max]
    SvtGpuCcsoParams *params; // [3] the planes' current parameters (device)
    uint8_t          *flags;  // [3][nb_max]
};

extern "C" int svtgpu_ccso_grid(int32_t width, int32_t height, int32_t plane, int32_t *nvfb, int32_t *nhfb) {
    if (width <= 0 || height <= 0 || plane < 0 || plane > 2 || !nvfb || !nhfb) return SVTGPU_ERR_INVALID_ARG;
    const Geo g = geo_of(width, height, plane);
    *nvfb = g.nvfb, *nhfb = g.nhfb;
    return SVTGPU_OK;
}

extern "C" int svtgpu_ccso_extend_luma(const void *luma, int32_t bits, int32_t stride, int32_t width, int32_t height,
                                       uint16_t *ext, void *stream) {
    if (!luma || !ext || width <= 0 || height <= 0 || stride < width || (bits != 8 && bits != 16))
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : svtgpu_default_stream();
    dim3        grid((width + 2 * PAD + 511) / 512, (height + 2 * PAD + 3) / 4);
    if (bits == 8) ccso_extend_kernel<uint8_t><<<grid, 256, 0, st>>>((const uint8_t *)luma, stride, width, height, ext);
    else ccso_extend_kernel<uint16_t><<<grid, 256, 0, st>>>((const uint16_t *)luma, stride, width, height, ext);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

extern "C" int svtgpu_ccso_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuCcsoState **out) {
    if (!ctx || !out || width < 16 || height < 16) return SVTGPU_ERR_INVALID_ARG;
    *out = nullptr;
    int nbp = 0, nb = 0;
    for (int p = 0; p < 3; p++) {
        const Geo g = geo_of(width, height, p);
        nbp = std::max(nbp, g.nbp), nb = std::max(nb, g.nb);
    }
    if (nb > MAXNB) return SVTGPU_ERR_UNSUPPORTED;
    SvtGpuCcsoState *s = new SvtGpuCcsoState();
    s->ctx = ctx, s->width = width, s->height = height, s->nbp_max = nbp, s->nb_max = nb;
    const size_t nbins = (size_t)3 * NKIND * nbp * NBIN, nmom = (size_t)3 * (NCOMBO + 1) * MOM_WORDS * nbp * NFINE;
    if (hipMalloc(&s->bins, nbins * sizeof(Bin)) != hipSuccess || hipMalloc(&s->mom, nmom * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&s->cost, 3 * NCFG * sizeof(double)) != hipSuccess ||
        hipMalloc(&s->lut, (size_t)3 * NCFG * NFINE) != hipSuccess ||
        hipMalloc(&s->ctrl, (size_t)3 * NCFG * nb) != hipSuccess ||
        hipMalloc(&s->params, 3 * sizeof(SvtGpuCcsoParams)) != hipSuccess ||
        hipMalloc(&s->flags, (size_t)3 * nb) != hipSuccess) {
        svtgpu_ccso_state_destroy(s);
        return SVTGPU_ERR_OOM;
    }
    if (hipMemset(s->params, 0, 3 * sizeof(SvtGpuCcsoParams)) != hipSuccess ||
        hipMemset(s->flags, 0, (size_t)3 * nb) != hipSuccess) {
        svtgpu_ccso_state_destroy(s);
        return SVTGPU_ERR_HIP;
    }
    *out = s;
    return SVTGPU_OK;
}

extern "C" void svtgpu_ccso_state_destroy(SvtGpuCcsoState *s) {
    if (!s) return;
    (void)hipFree(s->bins), (void)hipFree(s->mom), (void)hipFree(s->cost), (void)hipFree(s->lut);
    (void)hipFree(s->ctrl), (void)hipFree(s->params), (void)hipFree(s->flags);
    delete s;
}

namespace {
// the searches of planes [p0, p0 + n) in one launch per pass (their kernels are latency-bound: side by side they share
// the device instead of running one after another)
int launch_search(SvtGpuCcsoState *s, const uint16_t *ext, const uint16_t *const *org, const uint16_t *const *rec,
                  int p0, int n, int32_t bd, int32_t rdmult, hipStream_t st) {
    Planes a{};
    a.ext = ext, a.bd = bd, a.rdmult = rdmult, a.plane0 = p0;
    // measured (scripts/r6/ccso_perf.py, profiles/r06/ccso/strip_threshold.txt): 64-row workgroups halve the flushes of
    // the cell tile, which pays where the tiles are dense (10-bit: 0.94 -> 0.75 ms at 4K, 0.44 -> 0.37 at 1440p with 60
    // blocks a plane) and is about even at 8 bits (4K 0.86 either way); at 1080p (40 blocks) too few workgroups
    static const int forced = [] { // SVTGPU_CCSO_STRIP=32|64 (tests: the 64-row path on small pictures)
        const char *e = std::getenv("SVTGPU_CCSO_STRIP");
        return e && (std::atoi(e) == 32 || std::atoi(e) == 64) ? std::atoi(e) : 0;
    }();
    a.strip = forced ? forced : s->nbp_max >= (bd > 8 ? 56 : 96) ? 64 : 32;
    int gx = 0, gm = 0;
    for (int p = 0; p < 3; p++) {
        a.g[p]      = geo_of(s->width, s->height, p);
        a.org[p]    = p >= p0 && p < p0 + n ? org[p - p0] : nullptr;
        a.rec[p]    = p >= p0 && p < p0 + n ? rec[p - p0] : nullptr;
        a.bins[p]   = s->bins + (size_t)p * NKIND * s->nbp_max * NBIN;
        a.mom[p]    = s->mom + (size_t)p * (NCOMBO + 1) * MOM_WORDS * s->nbp_max * NFINE;
        a.cost[p]   = s->cost + (size_t)p * NCFG;
        a.lut[p]    = s->lut + (size_t)p * NCFG * NFINE;
        a.ctrl[p]   = s->ctrl + (size_t)p * NCFG * s->nb_max;
        a.params[p] = s->params + p;
        a.flags[p]  = s->flags + (size_t)p * s->nb_max;
        if (p >= p0 && p < p0 + n) gx = std::max(gx, a.g[p].nbp * (a.g[p].bs / a.strip)), gm = std::max(gm, a.g[p].nbp);
    }
    HIP_TRY(hipMemsetAsync(a.bins[p0], 0, (size_t)n * NKIND * s->nbp_max * NBIN * sizeof(Bin), st));
    ccso_bins_kernel<<<dim3(gx, NKIND, n), BTHREADS, 0, st>>>(a);
    HIP_TRY(hipGetLastError());
    ccso_merge_kernel<<<dim3(gm, NKIND, n), 256, 0, st>>>(a);
    HIP_TRY(hipGetLastError());
    ccso_train_kernel<<<dim3(NCFG, 1, n), TT, 0, st>>>(a);
    HIP_TRY(hipGetLastError());
    ccso_final_kernel<<<n, 256, 0, st>>>(a);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

int read_result(SvtGpuCcsoState *s, int plane, SvtGpuCcsoParams *params_out, uint8_t *flags_out, hipStream_t st) {
    const Geo g = geo_of(s->width, s->height, plane);
    if (params_out)
        HIP_TRY(hipMemcpyAsync(params_out, s->params + plane, sizeof(SvtGpuCcsoParams), hipMemcpyDeviceToHost, st));
    if (flags_out)
        HIP_TRY(hipMemcpyAsync(flags_out, s->flags + (size_t)plane * s->nb_max, g.nb, hipMemcpyDeviceToHost, st));
    svtgpu_count_xfer(1, (params_out ? sizeof(SvtGpuCcsoParams) : 0) + (flags_out ? g.nb : 0));
    return SVTGPU_OK;
}
} // namespace

extern "C" int svtgpu_ccso_search_plane(SvtGpuCcsoState *s, const uint16_t *ext, const uint16_t *org,
                                        const uint16_t *rec, int32_t plane, int32_t bit_depth, int32_t rdmult,
                                        SvtGpuCcsoParams *params_out, uint8_t *flags_out, void *stream) {
    if (!s || !ext || !org || !rec || plane < 0 || plane > 2 || bit_depth < 8 || bit_depth > 12 || rdmult < 0)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    if (int rc = launch_search(s, ext, &org, &rec, plane, 1, bit_depth, rdmult, st)) return rc;
    if (params_out || flags_out) {
        if (int rc = read_result(s, plane, params_out, flags_out, st)) return rc;
        HIP_TRY(hipStreamSynchronize(st));
    }
    return SVTGPU_OK;
}

extern "C" int svtgpu_ccso_search_frame(SvtGpuCcsoState *s, const uint16_t *ext, const uint16_t *const org[3],
                                        const uint16_t *const rec[3], int32_t bit_depth, int32_t rdmult,
                                        int32_t base_q_idx, SvtGpuCcsoParams params_out[3],
                                        uint8_t *const flags_out[3], int32_t *frame_flag, void *stream) {
    if (!s || !ext || !org || !rec || !frame_flag || bit_depth < 8 || bit_depth > 12 || rdmult < 0)
        return SVTGPU_ERR_INVALID_ARG;
    for (int p = 0; p < 3; p++)
        if (!org[p] || !rec[p]) return SVTGPU_ERR_INVALID_ARG;
    const int64_t r = (int64_t)rdmult * std::min(std::max(base_q_idx, 1), 63); // EbPickccso.c:788-793
    if (r >= INT_MAX) return 1;
    hipStream_t st = pick_stream(s->ctx, stream);
    if (int rc = launch_search(s, ext, org, rec, 0, 3, bit_depth, (int32_t)r, st)) return rc;
    *frame_flag = 0;
    if (!params_out) return SVTGPU_OK; // the result stays on the device (apply with params = NULL)
    for (int p = 0; p < 3; p++)
        if (int rc = read_result(s, p, &params_out[p], flags_out ? flags_out[p] : nullptr, st)) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    for (int p = 0; p < 3; p++) *frame_flag |= params_out[p].enable;
    return SVTGPU_OK;
}

extern "C" int svtgpu_ccso_apply_plane(SvtGpuCcsoState *s, const uint16_t *ext, int32_t plane, int32_t bit_depth,
                                       void *dst, int32_t dst_bits, int32_t dst_stride, const SvtGpuCcsoParams *params,
                                       const uint8_t *flags, void *stream) {
    if (!s || !ext || !dst || plane < 0 || plane > 2 || (dst_bits != 8 && dst_bits != 16) || bit_depth < 8 ||
        bit_depth > 12 || (params && !flags))
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    const Geo   g  = geo_of(s->width, s->height, plane);
    if (dst_stride < g.pw) return SVTGPU_ERR_INVALID_ARG;
    SvtGpuCcsoParams *dp = s->params + plane;
    uint8_t          *df = s->flags + (size_t)plane * s->nb_max;
    if (params) {
        if (params->max_band_log2 > 7 || params->quant_idx > 3 || params->ext_filter_support > 5 ||
            params->edge_clf > 1 || (!params->bo_only && params->max_band_log2 > 3))
            return SVTGPU_ERR_INVALID_ARG;
        HIP_TRY(hipMemcpyAsync(dp, params, sizeof(SvtGpuCcsoParams), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(df, flags, g.nb, hipMemcpyHostToDevice, st));
        svtgpu_count_xfer(0, sizeof(SvtGpuCcsoParams) + g.nb);
    }
    dim3 grid((g.pw + 63) / 64, (g.ph + 3) / 4);
    if (dst_bits == 8)
        ccso_apply_kernel<uint8_t><<<grid, 256, 0, st>>>(ext, (uint8_t *)dst, dst_stride, dp, df, g, bit_depth);
    else ccso_apply_kernel<uint16_t><<<grid, 256, 0, st>>>(ext, (uint16_t *)dst, dst_stride, dp, df, g, bit_depth);
    HIP_TRY(hipGetLastError());
    if (params) HIP_TRY(hipStreamSynchronize(st)); // the host params / flags may be reused once this returns
    return SVTGPU_OK;
}

// ---------------------------------------------------------------------------------------------
// per-block RTCD shims (common_dsp_rtcd.h:1025-1090): host pointers staged over the span each call touches
// ---------------------------------------------------------------------------------------------
namespace {
struct BlkArgs {
    int             mode; // 0 ccso_derive_src_block, 1 ccso_filter_block_hbd_with_buf, 2 ccso_filter_block_hbd_wo_buf
    const uint16_t *src;
    uint16_t       *dst;
    uint8_t        *cls0, *cls1;
    const int8_t   *lut;
    int32_t        *last_cls; // wo_buf: the classes of the last sample (the reference leaves them in src_cls)
    int src_stride, dst_stride, cls_stride, x, y_end, x_end, hs, vs, q, nq, loc0, loc1, maxv, shift, bo, single, clf;
};

__global__ __launch_bounds__(256) void ccso_block_kernel(BlkArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.y_end * a.x_end) return;
    const int       yp = i / a.x_end, xp = a.x + i % a.x_end;
    const uint16_t *c  = a.src + (ptrdiff_t)(yp << a.vs) * a.src_stride + (xp << a.hs);
    int             c0 = 0, c1 = 0;
    if (a.mode == 0 || (a.mode == 2 && !a.bo)) { // cal_filter_support (EbCcso.c:238-259)
        const int d0 = c[a.loc0] - c[0], d1 = c[a.loc1] - c[0];
        if (a.clf == 0) c0 = d0 > a.q ? 2 : d0 < a.nq ? 0 : 1, c1 = d1 > a.q ? 2 : d1 < a.nq ? 0 : 1;
        else c0 = d0 < a.nq ? 0 : 1, c1 = d1 < a.nq ? 0 : 1;
    }
    const ptrdiff_t ci = (ptrdiff_t)(yp << a.vs) * a.cls_stride + (xp << a.hs);
    if (a.mode == 0) {
        a.cls0[ci] = (uint8_t)c0, a.cls1[ci] = (uint8_t)c1;
        return;
    }
    if (a.mode == 1 && !a.bo) c0 = a.cls0[ci], c1 = a.cls1[ci];
    if (a.mode == 2 && i == a.y_end * a.x_end - 1) a.last_cls[0] = c0, a.last_cls[1] = c1;
    const int band = a.single ? 0 : c[0] >> a.shift;
    uint16_t *d    = a.dst + (ptrdiff_t)yp * a.dst_stride + xp;
    *d             = (uint16_t)clampi(a.lut[(band << 4) + (c0 << 2) + c1] + (int)*d, 0, a.maxv);
}

__global__ __launch_bounds__(256) void ccso_dist_kernel(const uint16_t *org, int os, const uint16_t *rec, int rs, int x,
                                                         int yo, int xo, unsigned long long *out) {
    unsigned long long ssd = 0;
    for (int i = threadIdx.x; i < yo * xo; i += 256) {
        const int e = org[(ptrdiff_t)os * (i / xo) + x + i % xo] - rec[(ptrdiff_t)rs * (i / xo) + x + i % xo];
        ssd += (unsigned long long)(e * e);
    }
    atomicAdd(out, ssd);
}

// a device copy of host [base + lo, base + hi) (element units); dev() = the device address of base
template <typename T> struct Span {
    T        *d = nullptr;
    ptrdiff_t lo = 0, n = 0;
    Span(const T *base, ptrdiff_t lo_, ptrdiff_t hi, hipStream_t st) : lo(lo_), n(hi - lo_) {
        HIP_OR_DIE(hipMalloc(&d, (size_t)n * sizeof(T)));
        HIP_OR_DIE(hipMemcpyAsync(d, base + lo, (size_t)n * sizeof(T), hipMemcpyHostToDevice, st));
    }
    T   *dev() const { return d - lo; }
    void back(T *base, hipStream_t st) const {
        HIP_OR_DIE(hipMemcpyAsync(base + lo, d, (size_t)n * sizeof(T), hipMemcpyDeviceToHost, st));
    }
    ~Span() { (void)hipFree(d); }
};

// the span [lo, hi) of the classifier's reads: every sample of the block and its two support neighbours
void src_span(const int *loc, bool neighbours, int stride, int x, int y_end, int x_end, int hs, int vs, ptrdiff_t *lo,
              ptrdiff_t *hi) {
    const int mn = neighbours ? std::min(0, std::min(loc[0], loc[1])) : 0;
    const int mx = neighbours ? std::max(0, std::max(loc[0], loc[1])) : 0;
    *lo          = (ptrdiff_t)(x << hs) + mn;
    *hi          = (ptrdiff_t)((y_end - 1) << vs) * stride + ((x + x_end - 1) << hs) + mx + 1;
}

void run_block(const BlkArgs &a, hipStream_t st) {
    ccso_block_kernel<<<(a.y_end * a.x_end + 255) / 256, 256, 0, st>>>(a);
    HIP_OR_DIE(hipGetLastError());
}
} // namespace

extern "C" uint64_t svtgpu_compute_distortion_block(const uint16_t *org, const int org_stride, const uint16_t *rec16,
                                                    const int rec_stride, const int x, const int y,
                                                    const int log2_filter_unit_size, const int height,
                                                    const int width) {
    const int bs = 1 << log2_filter_unit_size;
    const int yo = y + bs >= height ? height - y : bs, xo = x + bs >= width ? width - x : bs;
    if (yo <= 0 || xo <= 0) return 0;
    hipStream_t         st = svtgpu_shim_stream();
    Span<uint16_t>      so(org, x, (ptrdiff_t)org_stride * (yo - 1) + x + xo, st);
    Span<uint16_t>      sr(rec16, x, (ptrdiff_t)rec_stride * (yo - 1) + x + xo, st);
    unsigned long long *d_out, h_out = 0;
    HIP_OR_DIE(hipMalloc(&d_out, sizeof(d_out[0])));
    HIP_OR_DIE(hipMemsetAsync(d_out, 0, sizeof(d_out[0]), st));
    ccso_dist_kernel<<<1, 256, 0, st>>>(so.dev(), org_stride, sr.dev(), rec_stride, x, yo, xo, d_out);
    HIP_OR_DIE(hipGetLastError());
    HIP_OR_DIE(hipMemcpyAsync(&h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    (void)hipFree(d_out);
    return h_out;
}

extern "C" void svtgpu_ccso_derive_src_block(const uint16_t *src_y, uint8_t *const src_cls0, uint8_t *const src_cls1,
                                             const int src_y_stride, const int ccso_stride, const int x, const int y,
                                             const int pic_width, const int pic_height, const int y_uv_hscale,
                                             const int y_uv_vscale, const int qstep, const int neg_qstep,
                                             const int *src_loc, const int blk_size, const int edge_clf) {
    const int y_end = std::min(pic_height - y, blk_size), x_end = std::min(pic_width - x, blk_size);
    if (y_end <= 0 || x_end <= 0) return;
    hipStream_t st = svtgpu_shim_stream();
    ptrdiff_t   lo, hi, clo, chi;
    src_span(src_loc, true, src_y_stride, x, y_end, x_end, y_uv_hscale, y_uv_vscale, &lo, &hi);
    src_span(src_loc, false, ccso_stride, x, y_end, x_end, y_uv_hscale, y_uv_vscale, &clo, &chi);
    Span<uint16_t> s(src_y, lo, hi, st);
    Span<uint8_t>  c0(src_cls0, clo, chi, st), c1(src_cls1, clo, chi, st);
    BlkArgs a{};
    a.mode = 0, a.src = s.dev(), a.cls0 = c0.dev(), a.cls1 = c1.dev(), a.src_stride = src_y_stride;
    a.cls_stride = ccso_stride, a.x = x, a.y_end = y_end, a.x_end = x_end, a.hs = y_uv_hscale, a.vs = y_uv_vscale;
    a.q = (uint8_t)qstep, a.nq = neg_qstep, a.loc0 = src_loc[0], a.loc1 = src_loc[1], a.clf = edge_clf;
    run_block(a, st);
    c0.back(src_cls0, st), c1.back(src_cls1, st);
    HIP_OR_DIE(hipStreamSynchronize(st));
}

extern "C" void svtgpu_ccso_filter_block_hbd_with_buf(const uint16_t *src_y, uint16_t *dst_yuv, const uint8_t *src_cls0,
                                                      const uint8_t *src_cls1, const int src_y_stride,
                                                      const int dst_stride, const int ccso_stride, const int x,
                                                      const int y, const int pic_width, const int pic_height,
                                                      const int8_t *filter_offset, const int blk_size,
                                                      const int y_uv_hscale, const int y_uv_vscale, const int max_val,
                                                      const uint8_t shift_bits, const uint8_t ccso_bo_only) {
    const int y_end = std::min(pic_height - y, blk_size), x_end = std::min(pic_width - x, blk_size);
    if (y_end <= 0 || x_end <= 0) return;
    hipStream_t st = svtgpu_shim_stream();
    ptrdiff_t   lo, hi, clo, chi;
    src_span(nullptr, false, src_y_stride, x, y_end, x_end, y_uv_hscale, y_uv_vscale, &lo, &hi);
    src_span(nullptr, false, ccso_stride, x, y_end, x_end, y_uv_hscale, y_uv_vscale, &clo, &chi);
    Span<uint16_t> s(src_y, lo, hi, st), d(dst_yuv, x, (ptrdiff_t)(y_end - 1) * dst_stride + x + x_end, st);
    Span<int8_t>   l(filter_offset, 0, SVTGPU_CCSO_LUT, st);
    BlkArgs        a{};
    a.mode = 1, a.src = s.dev(), a.dst = d.dev(), a.lut = l.dev(), a.src_stride = src_y_stride;
    a.dst_stride = dst_stride, a.cls_stride = ccso_stride, a.x = x, a.y_end = y_end, a.x_end = x_end;
    a.hs = y_uv_hscale, a.vs = y_uv_vscale, a.maxv = max_val, a.shift = shift_bits, a.bo = ccso_bo_only;
    if (!ccso_bo_only) { // band-offset-only: the class buffers are not read (EbCcso.c:24-30)
        Span<uint8_t> k0(src_cls0, clo, chi, st), k1(src_cls1, clo, chi, st);
        a.cls0 = k0.dev(), a.cls1 = k1.dev();
        run_block(a, st);
        d.back(dst_yuv, st);
        HIP_OR_DIE(hipStreamSynchronize(st));
        return;
    }
    run_block(a, st);
    d.back(dst_yuv, st);
    HIP_OR_DIE(hipStreamSynchronize(st));
}

extern "C" void svtgpu_ccso_filter_block_hbd_wo_buf(const uint16_t *src_y, uint16_t *dst_yuv, const int x, const int y,
                                                    const int pic_width, const int pic_height, int *src_cls,
                                                    const int8_t *offset_buf, const int src_y_stride,
                                                    const int dst_stride, const int y_uv_hscale, const int y_uv_vscale,
                                                    const int thr, const int neg_thr, const int *src_loc,
                                                    const int max_val, const int blk_size, const bool isSingleBand,
                                                    const uint8_t shift_bits, const int edge_clf,
                                                    const uint8_t ccso_bo_only) {
    const int y_end = std::min(pic_height - y, blk_size), x_end = std::min(pic_width - x, blk_size);
    if (y_end <= 0 || x_end <= 0) return;
    hipStream_t st = svtgpu_shim_stream();
    ptrdiff_t   lo, hi;
    src_span(src_loc, !ccso_bo_only, src_y_stride, x, y_end, x_end, y_uv_hscale, y_uv_vscale, &lo, &hi);
    Span<uint16_t> s(src_y, lo, hi, st), d(dst_yuv, x, (ptrdiff_t)(y_end - 1) * dst_stride + x + x_end, st);
    Span<int8_t>   l(offset_buf, 0, SVTGPU_CCSO_LUT, st);
    Span<int32_t>  k(src_cls, 0, 2, st);
    BlkArgs        a{};
    a.mode = 2, a.src = s.dev(), a.dst = d.dev(), a.lut = l.dev(), a.last_cls = k.dev(), a.src_stride = src_y_stride;
    a.dst_stride = dst_stride, a.x = x, a.y_end = y_end, a.x_end = x_end, a.hs = y_uv_hscale, a.vs = y_uv_vscale;
    a.q = (uint8_t)thr, a.nq = neg_thr, a.loc0 = ccso_bo_only ? 0 : src_loc[0], a.loc1 = ccso_bo_only ? 0 : src_loc[1];
    a.maxv = max_val, a.shift = shift_bits, a.bo = ccso_bo_only, a.single = isSingleBand, a.clf = edge_clf;
    run_block(a, st);
    d.back(dst_yuv, st), k.back(src_cls, st);
    HIP_OR_DIE(hipStreamSynchronize(st));
}
