// lr_search.hip — loop-restoration parameter search on gfx950 (restoration_seg_search + rest_finish_search).
//
// Reference: Source/Lib/Encoder/Codec/EbRestorationPick.c (search :129-1460, finish :1555-1634), with the filters
// of Common/Codec/EbRestoration.c and convolve.c; the rate helpers of EbEntropyCoding.c:2876-3022.
//
// The search runs without stripe boundaries (use_boundaries_in_rest_search = 0, EbEncHandle.c:4162), so every
// filter output is a per-pixel function of the edge-clamped CDEF output.  The data-parallel work runs on the
// device over a tile list (<= 64x64 tiles aligned to each restoration unit):
//   unit_sums_kernel      Σ dgd (Wiener average) and the RESTORE_NONE SSE per unit
//   wiener_stats_kernel   the 7x7 (5x5, 3x3) Wiener statistics M, H of svt_av1_compute_stats: each lane
//                         accumulates a window-column pair block (49 MACs per 14 LDS reads) over a slice of the
//                         tile; per-tile partials are reduced per unit without atomics
//   wiener_trial_kernel   SSE of a unit filtered with candidate taps (one candidate per unit per launch)
//   sgr_flt_kernel        the self-guided filters of every searched ep (flt kept in HBM as int16) and the 2x2
//                         projection moments per (unit, ep) in exact int64
//   proj_err_kernel       projection error of candidate xqd per (unit, ep)
//   sgr_sse_kernel        SSE of the chosen self-guided unit output (with clipping)
// The sequential parts — the int64 fixed-point Wiener solve, the coordinate-descent refinements (advanced in
// lock-step rounds: all units / (unit, ep) pairs propose one candidate per launch) and the RD pass over the
// units — run on the host exactly as the reference orders them.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "lr_common.h"

namespace {

struct Tile {
    int32_t unit, x0, y0, w, h;
};
struct URect {
    int32_t h_start, h_end, v_start, v_end;
};

constexpr int PRJ_MIN0 = -96, PRJ_MAX0 = 31, PRJ_MIN1 = -32, PRJ_MAX1 = 95;
const int     kTapMin[3] = {-5, -23, -17}, kTapMax[3] = {10, 8, 46};
const int     kHostSgrR[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                              {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};

template <typename T>
__device__ inline int px(const T *p, int stride, int W, int H, int y, int x) {
    y = min(max(y, 0), H - 1);
    x = min(max(x, 0), W - 1);
    return p[(size_t)y * stride + x];
}

__device__ inline unsigned long long wave_sum(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

struct PlaneArgs {
    const void *dgd, *src;
    int32_t     dstride, sstride, W, H, bd;
    const Tile *tiles;
    const URect *units;
};

// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void unit_sums_kernel(const PlaneArgs a, unsigned long long *sum,
                                                        unsigned long long *sse) {
    const Tile t = a.tiles[blockIdx.x];
    const T   *d = (const T *)a.dgd, *s = (const T *)a.src;
    unsigned long long ps = 0, pe = 0;
    for (int i = threadIdx.x; i < t.w * t.h; i += 256) {
        const int y = t.y0 + i / t.w, x = t.x0 + i % t.w;
        const int dv = d[(size_t)y * a.dstride + x], sv = s[(size_t)y * a.sstride + x];
        ps += (unsigned)dv;
        pe += (unsigned long long)((dv - sv) * (dv - sv));
    }
    ps = wave_sum(ps);
    pe = wave_sum(pe);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&sum[t.unit], ps);
        atomicAdd(&sse[t.unit], pe);
    }
}

// ---------------------------------------------------------------------------------------------
// Wiener statistics: jobs = window-column pairs (c1 <= c2) + one M job; 8 lanes per job split the pixels
// ---------------------------------------------------------------------------------------------
constexpr int ST_APRON = 3, ST_W = 64 + 2 * ST_APRON;
template <typename T>
__global__ __launch_bounds__(256) void wiener_stats_kernel(const PlaneArgs a, int win, const unsigned long long *sum,
                                                           long long *part) {
    __shared__ int D[ST_W * ST_W];
    __shared__ int S[64 * 64];
    const Tile  t   = a.tiles[blockIdx.x];
    const URect u   = a.units[t.unit];
    const long long area = (long long)(u.h_end - u.h_start) * (u.v_end - u.v_start);
    const int   avg  = (int)(sum[t.unit] / (unsigned long long)area);
    const T    *d = (const T *)a.dgd, *s = (const T *)a.src;
    for (int i = threadIdx.x; i < (t.h + 6) * (t.w + 6); i += 256) {
        const int r = i / (t.w + 6), c = i % (t.w + 6);
        D[r * ST_W + c] = px(d, a.dstride, a.W, a.H, t.y0 + r - 3, t.x0 + c - 3) - avg;
    }
    for (int i = threadIdx.x; i < t.h * t.w; i += 256)
        S[(i / t.w) * 64 + i % t.w] = (int)s[(size_t)(t.y0 + i / t.w) * a.sstride + t.x0 + i % t.w] - avg;
    __syncthreads();
    const int half = win >> 1, npair = win * (win + 1) / 2, njob = npair + 1;
    const int job = threadIdx.x >> 3, g = threadIdx.x & 7;
    long long *out = part + (size_t)blockIdx.x * (size_t)njob * 49;
    int        acc[49];
#pragma unroll
    for (int k = 0; k < 49; k++) acc[k] = 0;
    if (job < npair) {
        int c1 = 0, rem = job; // job -> (c1, c2), c1 <= c2
        while (rem >= win - c1) rem -= win - c1, c1++;
        const int c2 = c1 + rem;
        for (int p = g; p < t.w * t.h; p += 8) {
            const int i = p / t.w, j = p % t.w;
            int       y1[7], y2[7];
#pragma unroll
            for (int r = 0; r < 7; r++)
                if (r < win) {
                    y1[r] = D[(i + 3 + r - half) * ST_W + j + 3 + c1 - half];
                    y2[r] = D[(i + 3 + r - half) * ST_W + j + 3 + c2 - half];
                }
#pragma unroll
            for (int r1 = 0; r1 < 7; r1++)
#pragma unroll
                for (int r2 = 0; r2 < 7; r2++)
                    if (r1 < win && r2 < win) acc[r1 * 7 + r2] += y1[r1] * y2[r2];
        }
    } else if (job == npair) { // M: y_k * x with k = c * win + r
        for (int p = g; p < t.w * t.h; p += 8) {
            const int i = p / t.w, j = p % t.w, x = S[i * 64 + j];
#pragma unroll
            for (int c = 0; c < 7; c++)
#pragma unroll
                for (int r = 0; r < 7; r++)
                    if (c < win && r < win) acc[c * 7 + r] += D[(i + 3 + r - half) * ST_W + j + 3 + c - half] * x;
        }
    }
    if (job <= npair) {
#pragma unroll
        for (int k = 0; k < 49; k++) {
            long long v = acc[k];
            v += __shfl_xor(v, 1, 64);
            v += __shfl_xor(v, 2, 64);
            v += __shfl_xor(v, 4, 64);
            if (g == 0) out[job * 49 + k] = v;
        }
    }
}

// per unit: sum the tile partials (tiles of a unit are contiguous in the tile list)
__global__ void reduce_parts_kernel(const long long *part, const int32_t *unit_tile0, int nvals, long long *out) {
    const int u = blockIdx.x, t0 = unit_tile0[u], t1 = unit_tile0[u + 1];
    for (int k = threadIdx.x; k < nvals; k += blockDim.x) {
        long long s = 0;
        for (int t = t0; t < t1; t++) s += part[(size_t)t * nvals + k];
        out[(size_t)u * nvals + k] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// Wiener trial: SSE of each active unit filtered with its candidate taps (hfilter[8], vfilter[8])
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void wiener_trial_kernel(const PlaneArgs a, const int16_t *taps,
                                                           const int32_t *active, unsigned long long *err) {
    __shared__ uint16_t v[(64 + 7) * (64 + 8)];
    __shared__ uint16_t tmp[(64 + 7) * 64];
    const Tile t = a.tiles[blockIdx.x];
    if (!active[t.unit]) return;
    const T  *d = (const T *)a.dgd, *s = (const T *)a.src;
    const int vs = 64 + 8;
    for (int i = threadIdx.x; i < (t.h + 7) * (t.w + 8); i += 256) {
        const int r = i / (t.w + 8), c = i % (t.w + 8);
        v[r * vs + c] = (uint16_t)px(d, a.dstride, a.W, a.H, t.y0 + r - 3, t.x0 + c - 3);
    }
    __syncthreads();
    const int16_t *hf = taps + t.unit * 16, *vf = hf + 8;
    const WienerRound rr  = wiener_round(a.bd);
    const int         lim = (1 << (a.bd + 1 + 7 - rr.r0)) - 1;
    for (int i = threadIdx.x; i < (t.h + 7) * t.w; i += 256) {
        const int       y = i / t.w, x = i % t.w;
        const uint16_t *p = v + y * vs + x;
        int             sum = ((int)p[3] << 7) + (1 << (a.bd + 6));
#pragma unroll
        for (int k = 0; k < 8; k++) sum += (int)p[k] * hf[k];
        tmp[y * 64 + x] = (uint16_t)min(max((sum + (1 << (rr.r0 - 1))) >> rr.r0, 0), lim);
    }
    __syncthreads();
    unsigned long long e = 0;
    const int          maxv = (1 << a.bd) - 1;
    for (int i = threadIdx.x; i < t.h * t.w; i += 256) {
        const int       y = i / t.w, x = i % t.w;
        const uint16_t *c = tmp + y * 64 + x;
        int             sum = ((int)c[3 * 64] << 7) - (1 << (a.bd + rr.r1 - 1));
#pragma unroll
        for (int k = 0; k < 8; k++) sum += (int)c[k * 64] * vf[k];
        const int o  = min(max((sum + (1 << (rr.r1 - 1))) >> rr.r1, 0), maxv);
        const int dd = o - (int)s[(size_t)(t.y0 + y) * a.sstride + t.x0 + x];
        e += (unsigned long long)(dd * dd);
    }
    e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) atomicAdd(&err[t.unit], e);
}

// ---------------------------------------------------------------------------------------------
// self-guided: flt0/flt1 of every searched ep, stored as int16, plus the projection moments
// mom[unit][ep] = {Σg1², Σg2², Σg1g2, Σg1·s, Σg2·s} with u = x<<4, s = (src<<4) - u, g = flt - u
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void sgr_flt_kernel(const PlaneArgs a, const int32_t *eps, int16_t *flt,
                                                      long long *mom, int nep_all) {
    __shared__ uint16_t v[(64 + 6) * (64 + 6)];
    __shared__ int      AB[2][66 * 66];
    const Tile t   = a.tiles[blockIdx.x];
    const int  ei  = blockIdx.y, ep = eps[ei];
    const T   *d = (const T *)a.dgd, *s = (const T *)a.src;
    const int  vs = 64 + 6, bw = t.w + 2;
    for (int i = threadIdx.x; i < (t.h + 6) * (t.w + 6); i += 256) {
        const int r = i / (t.w + 6), c = i % (t.w + 6);
        v[r * vs + c] = (uint16_t)px(d, a.dstride, a.W, a.H, t.y0 + r - 3, t.x0 + c - 3);
    }
    __syncthreads();
    const uint16_t *v0  = v + 3 * vs + 3;
    const size_t    pn  = (size_t)a.W * a.H;
    int16_t        *f0g = flt + (size_t)ei * 2 * pn, *f1g = f0g + pn;
    const int       r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
    constexpr int   PX = 64 * 64 / 256;
    int             f[2][PX]; // pixel k of this lane: threadIdx.x + k * 256
    for (int pass = 0; pass < 2; pass++) {
        const int r = pass ? r1 : r0;
        if (!r) continue;
        for (int i = threadIdx.x; i < (t.h + 2) * bw; i += 256) {
            const int y = i / bw - 1, x = i % bw - 1;
            if (r == 2 && !(y & 1)) continue;
            sgr_ab(v0, vs, y, x, r, c_sgr_s[ep][pass], a.bd, &AB[0][i], &AB[1][i]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PX; k++) {
            const int i = threadIdx.x + k * 256;
            if (i >= t.w * t.h) break;
            const int  y = i / t.w, x = i % t.w;
            const int *A = AB[0] + (y + 1) * bw + x + 1, *B = AB[1] + (y + 1) * bw + x + 1;
            int        aa, bb, nb;
            if (r == 1) {
                aa = (A[0] + A[-1] + A[1] + A[-bw] + A[bw]) * 4 + (A[-bw - 1] + A[bw - 1] + A[-bw + 1] + A[bw + 1]) * 3;
                bb = (B[0] + B[-1] + B[1] + B[-bw] + B[bw]) * 4 + (B[-bw - 1] + B[bw - 1] + B[-bw + 1] + B[bw + 1]) * 3;
                nb = 5;
            } else if (!(y & 1)) {
                aa = (A[-bw] + A[bw]) * 6 + (A[-bw - 1] + A[bw - 1] + A[-bw + 1] + A[bw + 1]) * 5;
                bb = (B[-bw] + B[bw]) * 6 + (B[-bw - 1] + B[bw - 1] + B[-bw + 1] + B[bw + 1]) * 5;
                nb = 5;
            } else {
                aa = A[0] * 6 + (A[-1] + A[1]) * 5;
                bb = B[0] * 6 + (B[-1] + B[1]) * 5;
                nb = 4;
            }
            const int sh = 8 + nb - 4;
            f[pass][k]   = (aa * (int)v0[y * vs + x] + bb + (1 << (sh - 1))) >> sh;
            (pass ? f1g : f0g)[(size_t)(t.y0 + y) * a.W + t.x0 + x] = (int16_t)f[pass][k];
        }
        __syncthreads();
    }
    // projection moments from the lane's own filter values
    long long m[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PX; k++) {
        const int i = threadIdx.x + k * 256;
        if (i >= t.w * t.h) break;
        const int y = i / t.w, x = i % t.w;
        const int u  = (int)v0[y * vs + x] << 4;
        const int sv = ((int)s[(size_t)(t.y0 + y) * a.sstride + t.x0 + x] << 4) - u;
        const int g1 = r0 > 0 ? f[0][k] - u : 0, g2 = r1 > 0 ? f[1][k] - u : 0;
        m[0] += (long long)g1 * g1;
        m[1] += (long long)g2 * g2;
        m[2] += (long long)g1 * g2;
        m[3] += (long long)g1 * sv;
        m[4] += (long long)g2 * sv;
    }
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const unsigned long long w = wave_sum((unsigned long long)m[k]);
        if ((threadIdx.x & 63) == 0) atomicAdd((unsigned long long *)&mom[((size_t)t.unit * nep_all + ei) * 5 + k], w);
    }
}

// projection error of candidate xq[unit][ep] = {xq0, xq1, active}
template <typename T>
__global__ __launch_bounds__(256) void proj_err_kernel(const PlaneArgs a, const int32_t *eps, const int16_t *flt,
                                                       const int32_t *cand, unsigned long long *err, int nep_all) {
    const Tile t  = a.tiles[blockIdx.x];
    const int  ei = blockIdx.y, ep = eps[ei];
    const int *c  = cand + ((size_t)t.unit * nep_all + ei) * 3;
    if (!c[2]) return;
    const int      xq0 = c[0], xq1 = c[1], r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
    const T       *d = (const T *)a.dgd, *s = (const T *)a.src;
    const size_t   pn = (size_t)a.W * a.H;
    const int16_t *f0 = flt + (size_t)ei * 2 * pn, *f1 = f0 + pn;
    unsigned long long e = 0;
    for (int i = threadIdx.x; i < t.w * t.h; i += 256) {
        const int    y = t.y0 + i / t.w, x = t.x0 + i % t.w;
        const size_t o = (size_t)y * a.W + x;
        const int    dv = d[(size_t)y * a.dstride + x], sv = s[(size_t)y * a.sstride + x];
        const int    u = dv << 4;
        int          v = 1 << 10;
        if (r0 > 0) v += xq0 * (f0[o] - u);
        if (r1 > 0) v += xq1 * (f1[o] - u);
        const int ee = (v >> 11) + dv - sv;
        e += (unsigned long long)((long long)ee * ee);
    }
    e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) atomicAdd(&err[(size_t)t.unit * nep_all + ei], e);
}

// SSE of the chosen self-guided output (apply_selfguided_restoration: projection, int16 wrap, clip)
template <typename T>
__global__ __launch_bounds__(256) void sgr_sse_kernel(const PlaneArgs a, const int16_t *flt, const int32_t *best,
                                                      unsigned long long *err) {
    const Tile t  = a.tiles[blockIdx.x];
    const int *b  = best + t.unit * 4; // {ep index, ep, xq0, xq1}
    const int  ei = b[0], ep = b[1], xq0 = b[2], xq1 = b[3], r0 = c_sgr_r[ep][0], r1 = c_sgr_r[ep][1];
    const T   *d = (const T *)a.dgd, *s = (const T *)a.src;
    const size_t   pn = (size_t)a.W * a.H;
    const int16_t *f0 = flt + (size_t)ei * 2 * pn, *f1 = f0 + pn;
    const int      maxv = (1 << a.bd) - 1;
    unsigned long long e = 0;
    for (int i = threadIdx.x; i < t.w * t.h; i += 256) {
        const int    y = t.y0 + i / t.w, x = t.x0 + i % t.w;
        const size_t o = (size_t)y * a.W + x;
        const int    dv = d[(size_t)y * a.dstride + x], sv = s[(size_t)y * a.sstride + x];
        const int    u = dv << 4;
        int          v = u << 7;
        if (r0 > 0) v += xq0 * (f0[o] - u);
        if (r1 > 0) v += xq1 * (f1[o] - u);
        const int16_t w  = (int16_t)((v + (1 << 10)) >> 11);
        const int     ov = min(max((int)w, 0), maxv);
        e += (unsigned long long)((ov - sv) * (ov - sv));
    }
    e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) atomicAdd(&err[t.unit], e);
}

// =============================================================================================
// host: the reference's sequential logic
// =============================================================================================
constexpr int64_t TAP_SCALE = (int64_t)1 << 16;
constexpr int     FILT_STEP = 128;

int wrap_index(int i, int win) { return i >= (win >> 1) + 1 ? win - 1 - i : i; }

int linsolve_wiener(int n, int64_t *A, int stride, int64_t *b, int32_t *x) { // EbRestorationPick.c:766-803
    for (int k = 0; k < n - 1; k++) {
        for (int i = n - 1; i > k; i--)
            if (std::llabs(A[(i - 1) * stride + k]) < std::llabs(A[i * stride + k])) {
                for (int j = 0; j < n; j++) std::swap(A[i * stride + j], A[(i - 1) * stride + j]);
                std::swap(b[i], b[i - 1]);
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

// update_a_sep_sym (solve_a) / update_b_sep_sym (EbRestorationPick.c:805-904); H viewed as hc[r][c]
void update_sep_sym(bool solve_b, int win, const int64_t *M, const int64_t *H, int32_t *a, int32_t *b) {
    const int win2 = win * win, h1 = (win >> 1) + 1;
    int64_t   A[4] = {0, 0, 0, 0}, B[16] = {0};
    int32_t   S[7];
    auto      hc = [&](int r, int c) { return H[(r / win) * win * win2 + (r % win) * win + c]; };
    if (!solve_b) {
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++) A[wrap_index(j, win)] += M[i * win + j] * b[i] / TAP_SCALE;
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++)
                for (int k = 0; k < win; k++)
                    for (int l = 0; l < win; l++)
                        B[wrap_index(l, win) * h1 + wrap_index(k, win)] +=
                            hc(j * win + i, k * win2 + l) * b[i] / TAP_SCALE * b[j] / TAP_SCALE;
    } else {
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++) A[wrap_index(i, win)] += M[i * win + j] * a[j] / TAP_SCALE;
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++)
                for (int k = 0; k < win; k++)
                    for (int l = 0; l < win; l++)
                        B[wrap_index(j, win) * h1 + wrap_index(i, win)] +=
                            hc(i * win + j, k * win2 + l) * a[k] / TAP_SCALE * a[l] / TAP_SCALE;
    }
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
        std::memcpy(solve_b ? b : a, S, win * sizeof(int32_t));
    }
}

void finalize_sym_filter(int win, const int32_t *f, int16_t *fi) { // EbRestorationPick.c:977-1006
    for (int i = 0; i < (win >> 1); i++) {
        const int64_t n = (int64_t)f[i] * FILT_STEP;
        fi[i]           = (int16_t)(n < 0 ? (n - TAP_SCALE / 2) / TAP_SCALE : (n + TAP_SCALE / 2) / TAP_SCALE);
    }
    auto clip = [](int v, int t) { return (int16_t)std::min(std::max(v, kTapMin[t]), kTapMax[t]); };
    if (win == 7) {
        fi[0] = clip(fi[0], 0), fi[1] = clip(fi[1], 1), fi[2] = clip(fi[2], 2);
    } else {
        fi[2] = clip(fi[1], 2), fi[1] = clip(fi[0], 1), fi[0] = 0;
    }
    fi[6] = fi[0], fi[5] = fi[1], fi[4] = fi[2];
    fi[3] = (int16_t)(-2 * (fi[0] + fi[1] + fi[2]));
    fi[7] = 0;
}

int64_t compute_score(int win, const int64_t *M, const int64_t *H, const int16_t *vf, const int16_t *hf) {
    int32_t   ab[49];
    int16_t   a[7], b[7];
    const int off = (7 - win) >> 1, win2 = win * win;
    a[3] = b[3] = FILT_STEP;
    for (int i = 0; i < 3; i++) {
        a[i] = a[6 - i] = vf[i];
        b[i] = b[6 - i] = hf[i];
        a[3] -= 2 * a[i];
        b[3] -= 2 * b[i];
    }
    for (int k = 0; k < win; k++)
        for (int l = 0; l < win; l++) ab[k * win + l] = a[l + off] * b[k + off];
    int64_t P = 0, Q = 0;
    for (int k = 0; k < win2; k++) {
        P += ab[k] * M[k] / FILT_STEP / FILT_STEP;
        for (int l = 0; l < win2; l++) Q += ab[k] * H[k * win2 + l] * ab[l] / FILT_STEP / FILT_STEP / FILT_STEP / FILT_STEP;
    }
    return (Q - 2 * P) - (H[(win2 >> 1) * win2 + (win2 >> 1)] - 2 * M[win2 >> 1]);
}

// rates (EbEntropyCoding.c:2876-3022, EbRestorationPick.c:655-668, 1008-1040)
int count_quniform(int n, int v) {
    if (n <= 1) return 0;
    const int l = 32 - __builtin_clz((unsigned)(n - 1)), m = (1 << l) - n;
    return v < m ? l - 1 : l;
}
int count_subexpfin(int n, int k, int v) {
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
int refsubexpfin(int n, int k, int ref, int v) {
    n &= 0xFFFF, ref &= 0xFFFF, v &= 0xFFFF;
    auto recenter = [](int r, int x) { return x > (r << 1) ? x : x >= r ? (x - r) << 1 : ((r - x) << 1) - 1; };
    const int rv = (ref << 1) <= n ? recenter(ref, v) : recenter(n - 1 - ref, n - 1 - v);
    return count_subexpfin(n, k, rv & 0xFFFF);
}
int wiener_bits(int win, const SvtGpuRestUnit &w, const SvtGpuRestUnit &ref) {
    static const int K[3] = {1, 2, 3};
    int              bits = 0;
    for (int f = 0; f < 2; f++) {
        const int16_t *a = f ? w.hfilter : w.vfilter, *r = f ? ref.hfilter : ref.vfilter;
        for (int t = win == 7 ? 0 : 1; t < 3; t++)
            bits += refsubexpfin(kTapMax[t] - kTapMin[t] + 1, K[t], r[t] - kTapMin[t], a[t] - kTapMin[t]);
    }
    return bits;
}
int sgrproj_bits(const SvtGpuRestUnit &s, const SvtGpuRestUnit &ref) {
    int bits = 4;
    if (kHostSgrR[s.ep][0] > 0) bits += refsubexpfin(PRJ_MAX0 - PRJ_MIN0 + 1, 4, ref.xqd[0] - PRJ_MIN0, s.xqd[0] - PRJ_MIN0);
    if (kHostSgrR[s.ep][1] > 0) bits += refsubexpfin(PRJ_MAX1 - PRJ_MIN1 + 1, 4, ref.xqd[1] - PRJ_MIN1, s.xqd[1] - PRJ_MIN1);
    return bits;
}
double rdcost(int rdmult, int64_t bits, int64_t sse) { // RDCOST_DBL (EbRestoration.h:346-347)
    return ((double)bits * rdmult) / (double)(1 << 9) + (double)sse * (1 << 7);
}

// Resumable coordinate descent shared by finer_tile_search_wiener_seg (EbRestorationPick.c:1042-1146) and
// finer_search_pixel_proj_error (:320-413): coordinates (f, p) move by -s then +s; at the first step size a
// successful move is repeated; a successful downward move ends the p loop of its filter.
struct Descent {
    int     start = 0, end = 1, nf = 1, p_lo = 0, p_hi = 0; // p in [p_lo, p_hi]
    bool    cont = true, skip_p[3] = {false, false, false};
    int     lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    int     val[2][3] = {{0, 0, 0}, {0, 0, 0}}; // coordinate values
    // state
    int     s = 0, f = 0, p = 0, phase = 0;      // phase 0: minus, 1: after minus, 2: plus
    bool    skip = false, init = true, done = false;
    int64_t err = 0;
    int     mf = 0, mp = 0, md = 0;              // pending move
    void    begin() { s = start, f = 0, p = p_lo, phase = 0, skip = false, init = true, done = false; }
    // proposes the next candidate (val holds it) or sets done; returns true when a candidate is pending
    bool next() {
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
            if (skip_p[p]) {
                p++;
                continue;
            }
            if (phase == 0) {
                if (val[f][p] - s >= lo[p]) {
                    val[f][p] -= s, mf = f, mp = p, md = -s;
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
            if (val[f][p] + s <= hi[p]) {
                val[f][p] += s, mf = f, mp = p, md = s;
                return true;
            }
            p++, phase = 0, skip = false;
        }
    }
    void report(int64_t e2) {
        if (init) {
            err = e2, init = false;
            return;
        }
        if (e2 > err) {
            val[mf][mp] -= md;
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

void set_wiener_taps(int16_t *t, const int *v) { // symmetric 7-tap from taps 0..2
    t[0] = t[6] = (int16_t)v[0];
    t[1] = t[5] = (int16_t)v[1];
    t[2] = t[4] = (int16_t)v[2];
    t[3] = (int16_t)(-2 * (v[0] + v[1] + v[2]));
    t[7] = 0;
}

struct DevBuf {
    void  *p = nullptr;
    size_t n = 0;
    int    get(size_t bytes) {
        if (bytes <= n) return SVTGPU_OK;
        if (p) (void)hipFree(p);
        p = nullptr, n = 0;
        HIP_TRY(hipMalloc(&p, bytes));
        n = bytes;
        return SVTGPU_OK;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

} // namespace

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

namespace {
template <typename T>
int search_plane(SvtGpuLrState *s, const SvtGpuFrame *rec, const SvtGpuFrame *src, int p,
                 const SvtGpuLrSearchControls *c, int *frame_type, SvtGpuLrUnitSearch *rec_out, hipStream_t st) {
    const int W = rec->pw[p], H = rec->ph[p], bd = rec->bit_depth;
    const int usz = s->unit_size[p], hu = s->hunits[p], vu = s->vunits[p], n = hu * vu;
    const int ext = usz * 3 / 2, off = 8 >> (p > 0);
    // units (foreach_rest_unit_in_tile, EbRestoration.c:1257-1294) and their <= 64x64 tiles
    std::vector<URect>   units;
    std::vector<Tile>    tiles;
    std::vector<int32_t> tile0;
    for (int y0 = 0; y0 < H;) {
        const int uh = (H - y0 < ext) ? H - y0 : usz;
        int       vs = std::max(0, y0 - off), ve = y0 + uh;
        if (ve < H) ve -= off;
        for (int x0 = 0; x0 < W;) {
            const int uw = (W - x0 < ext) ? W - x0 : usz;
            tile0.push_back((int)tiles.size());
            for (int y = vs; y < ve; y += 64)
                for (int x = x0; x < x0 + uw; x += 64)
                    tiles.push_back({(int)units.size(), x, y, std::min(64, x0 + uw - x), std::min(64, ve - y)});
            units.push_back({x0, x0 + uw, vs, ve});
            x0 += uw;
        }
        y0 += uh;
    }
    tile0.push_back((int)tiles.size());
    if ((int)units.size() != n) return SVTGPU_ERR_INVALID_ARG;
    const int nt = (int)tiles.size();
    // plane-sized scratch: tiles, units, accumulators, Wiener partials and candidates
    const int win_l = c->wn_filter_tap_lvl == 1 ? 7 : c->wn_filter_tap_lvl == 2 ? 5 : 3;
    const int win = p == 0 ? win_l : std::min(win_l, 5), nval = (win * (win + 1) / 2 + 1) * 49;
    std::vector<int32_t> eps;
    const int q = p > 0;
    if (c->sg_enabled && (!p || c->sg_use_chroma))
        for (int e = c->sg_start_ep[q]; e < c->sg_end_ep[q]; e += std::max(1, c->sg_ep_inc[q])) eps.push_back(e);
    const int ne = std::max(1, (int)eps.size());
    size_t    off_b = 0;
    auto      carve = [&](size_t bytes) {
        const size_t o = off_b;
        off_b += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_tiles = carve(sizeof(Tile) * nt), o_units = carve(sizeof(URect) * n), o_t0 = carve(4 * (n + 1));
    const size_t o_sum = carve(8 * n), o_sse = carve(8 * n), o_part = carve(8 * (size_t)nt * nval),
                 o_mh = carve(8 * (size_t)n * nval), o_taps = carve(2 * 16 * (size_t)n), o_act = carve(4 * (size_t)n),
                 o_err = carve(8 * (size_t)n * ne), o_eps = carve(4 * ne), o_mom = carve(8 * 5 * (size_t)n * ne),
                 o_cand = carve(4 * 3 * (size_t)n * ne), o_best = carve(4 * 4 * (size_t)n);
    if (off_b > s->work_bytes) {
        (void)hipFree(s->d_work);
        s->d_work = nullptr, s->work_bytes = 0;
        HIP_TRY(hipMalloc(&s->d_work, off_b));
        s->work_bytes = off_b;
    }
    if (!eps.empty() && !s->d_flt) HIP_TRY(hipMalloc(&s->d_flt, sizeof(int16_t) * 2 * 16 * (size_t)s->width * s->height));
    uint8_t *wb = (uint8_t *)s->d_work;
    auto     dp = [&](size_t o) { return (void *)(wb + o); };
    HIP_TRY(hipMemcpyAsync(dp(o_tiles), tiles.data(), sizeof(Tile) * nt, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dp(o_units), units.data(), sizeof(URect) * n, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(dp(o_t0), tile0.data(), 4 * (n + 1), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(dp(o_sum), 0, 8 * (size_t)n, st));
    HIP_TRY(hipMemsetAsync(dp(o_sse), 0, 8 * (size_t)n, st));
    PlaneArgs a;
    a.dgd = rec->plane[p], a.src = src->plane[p], a.dstride = rec->stride[p], a.sstride = src->stride[p];
    a.W = W, a.H = H, a.bd = bd, a.tiles = (const Tile *)dp(o_tiles), a.units = (const URect *)dp(o_units);
    hipLaunchKernelGGL(unit_sums_kernel<T>, dim3(nt), dim3(256), 0, st, a, (unsigned long long *)dp(o_sum),
                       (unsigned long long *)dp(o_sse));
    HIP_TRY(hipGetLastError());
    std::vector<uint64_t> h_sse(n);
    HIP_TRY(hipMemcpyAsync(h_sse.data(), dp(o_sse), 8 * n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<SvtGpuLrUnitSearch> rs(n);
    for (int u = 0; u < n; u++) {
        std::memset(&rs[u], 0, sizeof rs[u]);
        rs[u].sse[0] = (int64_t)h_sse[u];
        rs[u].sse[1] = INT64_MAX;
    }
    // ---------------- Wiener (search_wiener_seg, EbRestorationPick.c:1337-1419) ----------------
    if (c->wn_enabled && (!p || c->wn_use_chroma)) {
        hipLaunchKernelGGL(wiener_stats_kernel<T>, dim3(nt), dim3(256), 0, st, a, win,
                           (const unsigned long long *)dp(o_sum), (long long *)dp(o_part));
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(reduce_parts_kernel, dim3(n), dim3(256), 0, st, (const long long *)dp(o_part),
                           (const int32_t *)dp(o_t0), nval, (long long *)dp(o_mh));
        HIP_TRY(hipGetLastError());
        std::vector<int64_t> mh((size_t)n * nval);
        HIP_TRY(hipMemcpyAsync(mh.data(), dp(o_mh), 8 * mh.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const int            win2 = win * win, div = bd == 10 ? 4 : 1, half = win >> 1;
        std::vector<Descent> ds(n);
        std::vector<bool>    live(n, false);
        std::vector<SvtGpuRestUnit> wu(n);
        for (int u = 0; u < n; u++) {
            // assemble M[k] (k = col * win + row) and the full H from the column-pair blocks
            const int64_t *blk = mh.data() + (size_t)u * nval;
            int64_t        M[49], Hm[49 * 49];
            int            pair = 0;
            for (int c1 = 0; c1 < win; c1++)
                for (int c2 = c1; c2 < win; c2++, pair++)
                    for (int r1 = 0; r1 < win; r1++)
                        for (int r2 = 0; r2 < win; r2++) {
                            const int64_t v = blk[pair * 49 + r1 * 7 + r2] / div;
                            const int     k = c1 * win + r1, l = c2 * win + r2;
                            Hm[k * win2 + l] = v;
                            Hm[l * win2 + k] = v;
                        }
            for (int cc = 0; cc < win; cc++)
                for (int r = 0; r < win; r++) M[cc * win + r] = blk[pair * 49 + cc * 7 + r] / div;
            (void)half;
            // wiener_decompose_sep_sym (:906-935): start from the mid taps (centre incl. the implicit step)
            static const int init[7] = {3, -7, 15, 128 - 2 * (3 - 7 + 15), 15, -7, 3};
            const int        poff    = (7 - win) >> 1;
            int32_t          va[7], hb[7];
            for (int i = 0; i < win; i++) va[i] = hb[i] = (int32_t)(TAP_SCALE / FILT_STEP * init[i + poff]);
            for (int it = 1; it < 5; it++) {
                update_sep_sym(false, win, M, Hm, va, hb);
                update_sep_sym(true, win, M, Hm, va, hb);
            }
            SvtGpuRestUnit w;
            std::memset(&w, 0, sizeof w);
            w.type = SVTGPU_RESTORE_WIENER;
            finalize_sym_filter(win, va, w.vfilter);
            finalize_sym_filter(win, hb, w.hfilter);
            if (compute_score(win, M, Hm, w.vfilter, w.hfilter) > 0) continue; // sse stays INT64_MAX
            wu[u]        = w;
            Descent &d   = ds[u];
            d.start      = 4;
            d.end        = c->wn_use_refinement ? (c->wn_max_one_refinement_step ? 4 : 1) : 8; // 8: no refinement
            d.cont       = !c->wn_max_one_refinement_step;
            d.nf         = 2;
            d.p_lo       = (7 - win) >> 1;
            d.p_hi       = 2;
            for (int t = 0; t < 3; t++) {
                d.lo[t]     = kTapMin[t], d.hi[t] = kTapMax[t];
                d.val[0][t] = w.hfilter[t]; // f = 0: hfilter, f = 1: vfilter (the reference's order)
                d.val[1][t] = w.vfilter[t];
            }
            d.begin();
            live[u] = true;
        }
        // refinement rounds: every live unit evaluates one candidate per launch
        std::vector<int16_t> taps((size_t)16 * n);
        std::vector<int32_t> act(n);
        std::vector<uint64_t> e(n);
        for (;;) {
            int nact = 0;
            for (int u = 0; u < n; u++) {
                act[u] = 0;
                if (!live[u]) continue;
                if (!ds[u].next()) {
                    live[u] = false;
                    continue;
                }
                set_wiener_taps(&taps[16 * u], ds[u].val[0]);
                set_wiener_taps(&taps[16 * u + 8], ds[u].val[1]);
                act[u] = 1;
                nact++;
            }
            if (!nact) break;
            HIP_TRY(hipMemcpyAsync(dp(o_taps), taps.data(), 2 * taps.size(), hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemcpyAsync(dp(o_act), act.data(), 4 * n, hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemsetAsync(dp(o_err), 0, 8 * (size_t)n, st));
            hipLaunchKernelGGL(wiener_trial_kernel<T>, dim3(nt), dim3(256), 0, st, a, (const int16_t *)dp(o_taps),
                               (const int32_t *)dp(o_act), (unsigned long long *)dp(o_err));
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(e.data(), dp(o_err), 8 * n, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            for (int u = 0; u < n; u++)
                if (act[u]) ds[u].report((int64_t)e[u]);
        }
        for (int u = 0; u < n; u++) {
            if (!wu[u].type) continue;
            rs[u].sse[1] = ds[u].err;
            rs[u].wiener = wu[u];
            set_wiener_taps(rs[u].wiener.hfilter, ds[u].val[0]);
            set_wiener_taps(rs[u].wiener.vfilter, ds[u].val[1]);
        }
    }
    // ---------------- self-guided (search_sgrproj_seg / search_selfguided_restoration) ----------------
    if (!eps.empty()) {
        HIP_TRY(hipMemcpyAsync(dp(o_eps), eps.data(), 4 * ne, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(dp(o_mom), 0, 8 * 5 * (size_t)n * ne, st));
        hipLaunchKernelGGL(sgr_flt_kernel<T>, dim3(nt, ne), dim3(256), 0, st, a, (const int32_t *)dp(o_eps), s->d_flt,
                           (long long *)dp(o_mom), ne);
        HIP_TRY(hipGetLastError());
        std::vector<int64_t> mom((size_t)5 * n * ne);
        HIP_TRY(hipMemcpyAsync(mom.data(), dp(o_mom), 8 * mom.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<Descent> ds((size_t)n * ne);
        std::vector<int32_t> xqd0((size_t)2 * n * ne);
        for (int u = 0; u < n; u++)
            for (int k = 0; k < ne; k++) {
                // svt_get_proj_subspace_c (:417-500): the integer moments are exact doubles
                const int      ep = eps[k];
                const int64_t *m  = mom.data() + ((size_t)u * ne + k) * 5;
                const double   size = (double)((units[u].h_end - units[u].h_start) * (units[u].v_end - units[u].v_start));
                double         H00 = (double)m[0], H11 = (double)m[1], H01 = (double)m[2], C0 = (double)m[3], C1 = (double)m[4];
                H00 /= size, H01 /= size, H11 /= size;
                const double H10 = H01;
                C0 /= size, C1 /= size;
                int32_t xq[2] = {0, 0};
                if (kHostSgrR[ep][0] == 0) {
                    if (!(H11 < 1e-8)) xq[1] = (int32_t)std::rint(C1 / H11 * (1 << 7));
                } else if (kHostSgrR[ep][1] == 0) {
                    if (!(H00 < 1e-8)) xq[0] = (int32_t)std::rint(C0 / H00 * (1 << 7));
                } else {
                    const double det = H00 * H11 - H01 * H10;
                    if (!(det < 1e-8)) {
                        xq[0] = (int32_t)std::rint((H11 * C0 - H01 * C1) / det * (1 << 7));
                        xq[1] = (int32_t)std::rint((H00 * C1 - H10 * C0) / det * (1 << 7));
                    }
                }
                // encode_xq (:502-518)
                int xd[2];
                if (kHostSgrR[ep][0] == 0) {
                    xd[0] = 0;
                    xd[1] = std::min(std::max(128 - xq[1], PRJ_MIN1), PRJ_MAX1);
                } else if (kHostSgrR[ep][1] == 0) {
                    xd[0] = std::min(std::max(xq[0], PRJ_MIN0), PRJ_MAX0);
                    xd[1] = std::min(std::max(128 - xd[0], PRJ_MIN1), PRJ_MAX1);
                } else {
                    xd[0] = std::min(std::max(xq[0], PRJ_MIN0), PRJ_MAX0);
                    xd[1] = std::min(std::max(128 - xd[0] - xq[1], PRJ_MIN1), PRJ_MAX1);
                }
                Descent &d = ds[(size_t)u * ne + k];
                d.start = 2, d.end = c->sg_refine[q] ? 1 : 4, d.cont = true, d.nf = 1, d.p_lo = 0, d.p_hi = 1;
                d.lo[0] = PRJ_MIN0, d.hi[0] = PRJ_MAX0, d.lo[1] = PRJ_MIN1, d.hi[1] = PRJ_MAX1;
                d.skip_p[0] = kHostSgrR[ep][0] == 0;
                d.skip_p[1] = kHostSgrR[ep][1] == 0;
                d.val[0][0] = xd[0], d.val[0][1] = xd[1];
                d.begin();
            }
        std::vector<int32_t>  cand((size_t)3 * n * ne);
        std::vector<uint64_t> e((size_t)n * ne);
        for (;;) {
            int nact = 0;
            for (size_t i = 0; i < ds.size(); i++) {
                cand[3 * i + 2] = 0;
                if (ds[i].done || !ds[i].next()) continue;
                const int ep = eps[i % ne];
                // svt_decode_xq (EbRestoration.c:634-646)
                const int x0 = ds[i].val[0][0], x1 = ds[i].val[0][1];
                cand[3 * i]     = kHostSgrR[ep][0] == 0 ? 0 : x0;
                cand[3 * i + 1] = kHostSgrR[ep][0] == 0 ? 128 - x1 : kHostSgrR[ep][1] == 0 ? 0 : 128 - x0 - x1;
                cand[3 * i + 2] = 1;
                nact++;
            }
            if (!nact) break;
            HIP_TRY(hipMemcpyAsync(dp(o_cand), cand.data(), 4 * cand.size(), hipMemcpyHostToDevice, st));
            HIP_TRY(hipMemsetAsync(dp(o_err), 0, 8 * e.size(), st));
            hipLaunchKernelGGL(proj_err_kernel<T>, dim3(nt, ne), dim3(256), 0, st, a, (const int32_t *)dp(o_eps),
                               (const int16_t *)s->d_flt, (const int32_t *)dp(o_cand),
                               (unsigned long long *)dp(o_err), ne);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(e.data(), dp(o_err), 8 * e.size(), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            for (size_t i = 0; i < ds.size(); i++)
                if (cand[3 * i + 2]) ds[i].report((int64_t)e[i]);
        }
        // best ep per unit (strict <, first), then the SSE of its clipped output
        std::vector<int32_t> best((size_t)4 * n);
        for (int u = 0; u < n; u++) {
            int64_t be = -1;
            int     bk = 0;
            for (int k = 0; k < ne; k++) {
                const int64_t err = ds[(size_t)u * ne + k].err;
                if (be == -1 || err < be) be = err, bk = k;
            }
            const Descent &d  = ds[(size_t)u * ne + bk];
            const int      ep = eps[bk];
            SvtGpuRestUnit g;
            std::memset(&g, 0, sizeof g);
            g.type = SVTGPU_RESTORE_SGRPROJ, g.ep = ep, g.xqd[0] = d.val[0][0], g.xqd[1] = d.val[0][1];
            rs[u].sgrproj  = g;
            best[4 * u]     = bk;
            best[4 * u + 1] = ep;
            best[4 * u + 2] = kHostSgrR[ep][0] == 0 ? 0 : g.xqd[0];
            best[4 * u + 3] = kHostSgrR[ep][0] == 0 ? 128 - g.xqd[1] : kHostSgrR[ep][1] == 0 ? 0 : 128 - g.xqd[0] - g.xqd[1];
        }
        HIP_TRY(hipMemcpyAsync(dp(o_best), best.data(), 4 * best.size(), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(dp(o_err), 0, 8 * (size_t)n, st));
        hipLaunchKernelGGL(sgr_sse_kernel<T>, dim3(nt), dim3(256), 0, st, a, (const int16_t *)s->d_flt,
                           (const int32_t *)dp(o_best), (unsigned long long *)dp(o_err));
        HIP_TRY(hipGetLastError());
        std::vector<uint64_t> es(n);
        HIP_TRY(hipMemcpyAsync(es.data(), dp(o_err), 8 * n, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int u = 0; u < n; u++) rs[u].sse[2] = (int64_t)es[u];
    }
    // ---------------- rest_finish_search (EbRestorationPick.c:1555-1634) ----------------
    const bool wn_on = c->wn_enabled && (!p || c->wn_use_chroma), sg_on = !eps.empty();
    const int  force = c->wn_enabled ? (c->sg_enabled ? 4 : 1) : (c->sg_enabled ? 2 : 0);
    const int  nrt   = n > 1 ? 4 : 3;
    std::vector<int>            brt((size_t)3 * n, 0);
    std::vector<SvtGpuRestUnit> uw(n), us(n);
    double                      best_cost = 0;
    int                         best_type = 0;
    static const int16_t        kMid[7]   = {3, -7, 15, -22, 15, -7, 3}; // set_default_wiener
    for (int r = 0; r < nrt; r++) {
        if (force != 4 && r != 0 && r != force) continue;
        if (p && ((r == 1 && !c->wn_use_chroma) || (r == 2 && !c->sg_use_chroma))) continue;
        SvtGpuRestUnit refw, refs;
        std::memset(&refw, 0, sizeof refw);
        std::memset(&refs, 0, sizeof refs);
        for (int k = 0; k < 7; k++) refw.vfilter[k] = refw.hfilter[k] = kMid[k];
        refs.xqd[0] = (PRJ_MIN0 + PRJ_MAX0) / 2, refs.xqd[1] = (PRJ_MIN1 + PRJ_MAX1) / 2;
        int64_t sse = 0, bits = 0;
        for (int u = 0; u < n; u++) {
            const SvtGpuLrUnitSearch &R = rs[u];
            if (r == 0) {
                sse += R.sse[0];
            } else if (r == 1) { // search_wiener_finish
                const int64_t bn = c->wiener_restore_cost[0];
                if (R.sse[1] == INT64_MAX) {
                    bits += bn, sse += R.sse[0], brt[3 * u] = 0;
                    continue;
                }
                uw[u]            = R.wiener;
                const int64_t bw = c->wiener_restore_cost[1] + ((int64_t)wiener_bits(win, R.wiener, refw) << 9);
                const bool    t  = rdcost(c->rdmult, bw >> 4, R.sse[1]) < rdcost(c->rdmult, bn >> 4, R.sse[0]);
                brt[3 * u]       = t ? 1 : 0;
                sse += R.sse[t ? 1 : 0];
                bits += t ? bw : bn;
                if (t) refw = R.wiener;
            } else if (r == 2) { // search_sgrproj_finish
                us[u]            = R.sgrproj;
                const int64_t bn = c->sgrproj_restore_cost[0];
                const int64_t bs = c->sgrproj_restore_cost[1] + ((int64_t)sgrproj_bits(R.sgrproj, refs) << 9);
                const bool    t  = rdcost(c->rdmult, bs >> 4, R.sse[2]) < rdcost(c->rdmult, bn >> 4, R.sse[0]);
                brt[3 * u + 1]   = t ? 2 : 0;
                sse += R.sse[t ? 2 : 0];
                bits += t ? bs : bn;
                if (t) refs = R.sgrproj;
            } else { // search_switchable (7 / 5 Wiener taps by plane)
                double  bc = 0;
                int64_t bb = 0;
                int     bt = 0;
                for (int t = 0; t < 3; t++) {
                    if (t > 0 && brt[3 * u + t - 1] == 0) continue;
                    const int64_t cp = t == 1 ? wiener_bits(p == 0 ? 7 : 5, uw[u], refw) : t == 2 ? sgrproj_bits(us[u], refs) : 0;
                    const int64_t b  = c->switchable_restore_cost[t] + (cp << 9);
                    const double  cost = rdcost(c->rdmult, b >> 4, R.sse[t]);
                    if (t == 0 || cost < bc) bc = cost, bb = b, bt = t;
                }
                brt[3 * u + 2] = bt;
                sse += R.sse[bt];
                bits += bb;
                if (bt == 1) refw = uw[u];
                if (bt == 2) refs = us[u];
            }
        }
        const double cost = rdcost(c->rdmult, bits >> 4, sse);
        if (r == 0 || cost < best_cost) best_cost = cost, best_type = r;
    }
    (void)wn_on, (void)sg_on;
    *frame_type = best_type;
    std::vector<SvtGpuRestUnit> out(n);
    for (int u = 0; u < n; u++) { // copy_unit_info
        std::memset(&out[u], 0, sizeof out[u]);
        if (best_type) {
            const int t = brt[3 * u + best_type - 1];
            out[u]      = t == 1 ? uw[u] : us[u];
            out[u].type = t;
        }
        if (rec_out) rec_out[u] = rs[u];
    }
    HIP_TRY(hipMemcpyAsync(s->d_units[p], out.data(), sizeof(SvtGpuRestUnit) * n, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}
} // namespace

extern "C" int svtgpu_lr_search_frame(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                      const SvtGpuLrSearchControls *ctrls, int32_t frame_type_out[3],
                                      SvtGpuLrUnitSearch *const search_out[3], void *stream) {
    if (!s || !recon || !source || !ctrls || !frame_type_out || recon->width != s->width ||
        recon->height != s->height || source->width != s->width || source->height != s->height ||
        recon->bit_depth != source->bit_depth)
        return SVTGPU_ERR_INVALID_ARG;
    if (recon->bit_depth != 8 && recon->bit_depth != 10) return SVTGPU_ERR_UNSUPPORTED;
    for (int q = 0; q < 2; q++)
        if (ctrls->sg_enabled && (ctrls->sg_start_ep[q] < 0 || ctrls->sg_end_ep[q] > 16 || ctrls->sg_ep_inc[q] < 1))
            return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st        = pick_stream(s->ctx, stream);
    const int   plane_end = ((ctrls->wn_enabled && ctrls->wn_use_chroma) || (ctrls->sg_enabled && ctrls->sg_use_chroma)) ? 2 : 0;
    for (int p = 0; p < 3; p++) frame_type_out[p] = SVTGPU_RESTORE_NONE;
    for (int p = 0; p <= plane_end; p++) {
        int rc = recon->bytes_per_sample == 2
            ? search_plane<uint16_t>(s, recon, source, p, ctrls, &frame_type_out[p], search_out ? search_out[p] : nullptr, st)
            : search_plane<uint8_t>(s, recon, source, p, ctrls, &frame_type_out[p], search_out ? search_out[p] : nullptr, st);
        if (rc) return rc;
    }
    return SVTGPU_OK;
}
