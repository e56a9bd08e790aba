// lr.hip — AV1 loop restoration (Wiener / self-guided) on gfx950: frame apply and RTCD shims.
//
// Reference (Source/Lib/): Common/Codec/convolve.c:109-232 (Wiener convolve add src),
// Common/Codec/EbRestoration.c:466-991 (box sums, self-guided filters, decode_xq, projection),
// :222-435 + :1067-1139 (processing stripes, boundary substitution), :1179-1296 (units of the frame),
// :1522-1680 (stripe boundary lines saved after deblocking / CDEF).
//
// Design (MI355X): a restoration unit's output at a pixel depends only on a 7x7 (Wiener) / 5x5+3x3
// (self-guided) window of its processing stripe's *virtual input*: the CDEF output rows of the stripe, the
// three rows above/below replaced by the saved deblocked lines (L0 L0 L1 / B0 B1 B1) inside the frame and by
// the replicated edge row at the frame top/bottom, and edge-replicated columns.  So the frame is processed
// as independent tiles of one stripe x 64 (luma) / 32 (chroma) columns — which never straddle a unit — one
// workgroup each: the virtual tile is staged in LDS straight from the resident DLF and CDEF frames (no line
// buffers, no frame extension pass), then the unit's filter runs from LDS and the tile is written once.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lr_common.h"

namespace {

// A, B of one self-guided pass at the centres (ys + YS m, x), m < ncent, x = -1 .. w (box radius R): an item slides a
// window of per-row sums down one column segment -- 2R + 1 row sums to start, YS more per further centre -- instead
// of reading the (2R + 1)^2 box at every centre (r = 2: 125 LDS reads per 11 centres instead of 275).  A and B land
// packed in one word, A | B << 9 (A <= 256; B < 2^20 up to 12 bits): one LDS array, so a tile takes 29 KB instead of
// 46 and five workgroups fit a CU instead of three
template <int R, int YS>
__device__ __forceinline__ void sgr_ab_slide(const uint16_t *v, int vs, int bw, int ys, int ncent, int s, int bd,
                                             uint32_t *P) {
    constexpr int N = 2 * R + 1;
    const int     G = max(1, NTHR / bw), per = (ncent + G - 1) / G; // column segments of `per` centres
    for (int it = threadIdx.x; it < bw * G; it += NTHR) {
        const int g = it / bw, x = it - g * bw - 1, m0 = g * per, m1 = min(ncent, m0 + per);
        if (m0 >= m1) continue;
        int  ws[N], wq[N];
        auto row = [&](int y, int &sum, int &sq) {
            const uint16_t *p = v + y * vs + x - R;
            sum = 0, sq = 0;
#pragma unroll
            for (int k = 0; k < N; k++) {
                const int q = p[k];
                sum += q, sq += q * q;
            }
        };
#pragma unroll
        for (int k = 0; k < N; k++) row(ys + YS * m0 - R + k, ws[k], wq[k]);
        for (int m = m0; m < m1; m++) {
            const int y = ys + YS * m;
            if (m > m0) {
#pragma unroll
                for (int k = 0; k + YS < N; k++) ws[k] = ws[k + YS], wq[k] = wq[k + YS];
#pragma unroll
                for (int k = N - YS; k < N; k++) row(y - R + k, ws[k], wq[k]);
            }
            int sum = 0, sq = 0;
#pragma unroll
            for (int k = 0; k < N; k++) sum += ws[k], sq += wq[k];
            int a, b;
            sgr_ab_from_sums(sum, sq, N * N, s, bd, c_x_by_xplus1, &a, &b);
            P[(y + 1) * bw + x + 1] = (uint32_t)a | ((uint32_t)b << 9);
        }
    }
}

// self-guided filter + projection (svt_apply_selfguided_restoration_c) of a w x h tile; P holds the packed A, B of
// (h+2) x (w+2) positions; flt0 is kept per thread between the passes (px k of thread = threadIdx.x + k * NTHR)
constexpr int SGR_MAXPX = 64 * 64 / NTHR;
template <typename T>
__device__ void sgr_tile(const uint16_t *v, int vs, uint32_t *P, int w, int h, int eps, const int32_t *xqd, int bd,
                         T *out, size_t os) {
    const int     bw = w + 2;
    const FastDiv dw(w);
    auto          pa = [](uint32_t p) { return (int)(p & 511u); };
    auto          pb = [](uint32_t p) { return (int)(p >> 9); };
    int           f0[SGR_MAXPX];
    const int     r0 = c_sgr_r[eps][0], r1 = c_sgr_r[eps][1];
    if (r0 > 0) { // r = 2 on odd rows -1, 1, 3, ...
        sgr_ab_slide<2, 2>(v, vs, bw, -1, (h + 3) / 2, c_sgr_s[eps][0], bd, P);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SGR_MAXPX; k++) {
            const int i = threadIdx.x + k * NTHR;
            if (i >= w * h) break;
            const int y = dw(i), x = i - y * w;
            const uint32_t *q = P + (y + 1) * bw + x + 1;
            int             aa, bb, nb;
            if (!(y & 1)) {
                const uint32_t n0 = q[-bw], n1 = q[bw], c0 = q[-bw - 1], c1 = q[bw - 1], c2 = q[-bw + 1], c3 = q[bw + 1];
                aa = (pa(n0) + pa(n1)) * 6 + (pa(c0) + pa(c1) + pa(c2) + pa(c3)) * 5;
                bb = (pb(n0) + pb(n1)) * 6 + (pb(c0) + pb(c1) + pb(c2) + pb(c3)) * 5;
                nb = 5;
            } else {
                const uint32_t m = q[0], l = q[-1], r = q[1];
                aa = pa(m) * 6 + (pa(l) + pa(r)) * 5;
                bb = pb(m) * 6 + (pb(l) + pb(r)) * 5;
                nb = 4;
            }
            const int sh = 8 + nb - 4;
            f0[k]        = (aa * (int)v[y * vs + x] + bb + (1 << (sh - 1))) >> sh;
        }
        __syncthreads();
    }
    if (r1 > 0) {
        sgr_ab_slide<1, 1>(v, vs, bw, -1, h + 2, c_sgr_s[eps][1], bd, P);
        __syncthreads();
    }
    // projection: xq from xqd (svt_decode_xq, EbRestoration.c:634-646)
    int xq0, xq1;
    if (r0 == 0)
        xq0 = 0, xq1 = 128 - xqd[1];
    else if (r1 == 0)
        xq0 = xqd[0], xq1 = 0;
    else
        xq0 = xqd[0], xq1 = 128 - xqd[0] - xqd[1];
    const int maxv = (1 << bd) - 1;
#pragma unroll
    for (int k = 0; k < SGR_MAXPX; k++) {
        const int i = threadIdx.x + k * NTHR;
        if (i >= w * h) break;
        const int y = dw(i), x = i - y * w;
        const int u = (int)v[y * vs + x] << 4;
        int       val = u << 7;
        if (r0 > 0) val += xq0 * (f0[k] - u);
        if (r1 > 0) {
            const uint32_t *q = P + (y + 1) * bw + x + 1;
            const uint32_t  e0 = q[0], e1 = q[-1], e2 = q[1], e3 = q[-bw], e4 = q[bw];
            const uint32_t  c0 = q[-bw - 1], c1 = q[bw - 1], c2 = q[-bw + 1], c3 = q[bw + 1];
            const int aa = (pa(e0) + pa(e1) + pa(e2) + pa(e3) + pa(e4)) * 4 + (pa(c0) + pa(c1) + pa(c2) + pa(c3)) * 3;
            const int bb = (pb(e0) + pb(e1) + pb(e2) + pb(e3) + pb(e4)) * 4 + (pb(c0) + pb(c1) + pb(c2) + pb(c3)) * 3;
            const int  f1 = (aa * (int)v[y * vs + x] + bb + (1 << 8)) >> 9;
            val += xq1 * (f1 - u);
        }
        const int16_t o = (int16_t)((val + (1 << 10)) >> 11);
        out[y * os + x] = (T)min(max((int)o, 0), maxv);
    }
}

// ---------------------------------------------------------------------------------------------
// frame apply: one workgroup per (stripe, column chunk) of a plane
// ---------------------------------------------------------------------------------------------
constexpr int TW = 64, TH = 64;
constexpr int VC0 = 8;                // virtual tile column 0 at LDS column 8 (16-B aligned rows and interior)
constexpr int VS  = VC0 + TW + 8;     // virtual tile columns -3 .. TW+4
constexpr int VR  = TH + 7;           // virtual tile rows -3 .. TH+3
struct LrPlaneArgs {
    const void           *dlf, *cdef;
    void                 *out;
    int32_t               dlf_stride, cdef_stride, out_stride;
    int32_t               W, H, ss, unit_size, hunits, vunits, nchunks, bd;
    int32_t               k0, c0, nc; // the (stripe, column chunk) tiles written: k0 + i / nc, c0 + i % nc
    int32_t               count;      // nk x nc tiles (the plane's block range is padded to a multiple of 8)
    const SvtGpuRestUnit *units;
};

// the filtered planes of one frame in one launch: the planes' tile grids back to back (fewer launch boundaries and
// one tail instead of three for a kernel of ~20 us per plane)
struct LrApplyArgs {
    LrPlaneArgs pl[3];
    int32_t     nplanes, end[3]; // end[i]: first block past plane i of the launch (each range a multiple of 8)
};

template <typename T>
__global__ __launch_bounds__(NTHR) void lr_apply_kernel(const LrApplyArgs args) {
    int pi = 0;
    while (pi + 1 < args.nplanes && (int)blockIdx.x >= args.end[pi]) pi++;
    const LrPlaneArgs &a = args.pl[pi];
    // XCD-aware order within each plane (its block range starts on a multiple of 8): every XCD takes a contiguous
    // eighth of each plane -- a few stripes, so the apron lines a tile shares with its neighbours (3 + 5 columns,
    // 7 rows) are fetched into one L2 instead of up to three, and the luma / chroma work stays spread over all XCDs
    const int b0  = pi ? args.end[pi - 1] : 0;
    const int blk = xcd_swizzle((int)blockIdx.x - b0, args.end[pi] - b0);
    if (blk >= a.count) return; // the padding to a multiple of 8
    __shared__ __attribute__((aligned(16))) uint16_t v[VR * VS];
    // a unit is Wiener or self-guided: the Wiener intermediate (VR x TW u16) shares the A/B arrays' LDS
    __shared__ uint32_t AB[(TH + 2) * (TW + 2)];
    static_assert(VR * TW * 2 <= sizeof(uint32_t) * (TH + 2) * (TW + 2), "Wiener intermediate in AB");
    uint16_t *t = (uint16_t *)AB;
    const int S = 64 >> a.ss, off = 8 >> a.ss, cwmax = 64 >> a.ss;
    const int k = a.k0 + blk / a.nc, c = a.c0 + blk % a.nc;
    const int y0 = max(0, k * S - off), y1 = min((k + 1) * S - off, a.H);
    const int x0 = c * cwmax, w = min(cwmax, a.W - x0), h = y1 - y0;
    if (h <= 0 || w <= 0) return;
    const int ur = min((y0 + off) / a.unit_size, a.vunits - 1), uc = min(x0 / a.unit_size, a.hunits - 1);
    const SvtGpuRestUnit u = a.units[ur * a.hunits + uc];
    const T *cdef = (const T *)a.cdef, *dlf = (const T *)a.dlf;
    T       *out  = (T *)a.out;
    const int segs = (w + 7) >> 3, lseg = cwmax == 64 ? 3 : 2; // 8-sample row segments (w is a multiple of 4)
    if (u.type == SVTGPU_RESTORE_NONE) { // copy: one vector load / store per segment
        for (int i = threadIdx.x; i < h << lseg; i += NTHR) {
            const int y = i >> lseg, sg = i & ((1 << lseg) - 1), x = x0 + 8 * sg;
            if (sg >= segs) continue;
            const T *src = cdef + (size_t)(y0 + y) * a.cdef_stride + x;
            T       *dst = out + (size_t)(y0 + y) * a.out_stride + x;
            if (x + 8 <= x0 + w) {
                if constexpr (sizeof(T) == 2) *(uint4 *)dst = *(const uint4 *)src;
                else *(uint2 *)dst = *(const uint2 *)src;
            } else {
                for (int j = 0; j < x0 + w - x; j++) dst[j] = src[j];
            }
        }
        return;
    }
    // virtual stripe input (svt_aom_setup_processing_stripe_boundary with saved lines, EbRestoration.c:271-352):
    // the source row of each virtual row, then the row's interior as 8-sample vector loads (all issued before the
    // LDS stores) and its 3 + 5 apron columns (edge-replicated) one sample each
    const int copy_above = y0 != 0;
    const int copy_below = !(y0 + S - (y0 == 0 ? off : 0) >= a.H);
    auto row_of = [&](int r) -> const T * {
        if (r < 0 && copy_above) return dlf + (size_t)(y0 + (r == -1 ? -1 : -2)) * a.dlf_stride;
        if (r >= h && r < h + 3 && copy_below) return dlf + (size_t)min(y1 + (r == h ? 0 : 1), a.H - 1) * a.dlf_stride;
        return cdef + (size_t)min(max(y0 + r, 0), a.H - 1) * a.cdef_stride;
    };
    constexpr int IT = (VR * 8 + NTHR - 1) / NTHR;
    uint4         seg[IT];
#pragma unroll
    for (int q = 0; q < IT; q++) {
        const int i = threadIdx.x + q * NTHR, r = (i >> lseg) - 3, sg = i & ((1 << lseg) - 1), x = x0 + 8 * sg;
        if (r >= h + 4 || sg >= segs) continue;
        const T *src = row_of(r) + x;
        if (x + 8 <= a.W) {
            if constexpr (sizeof(T) == 2) {
                seg[q] = *(const uint4 *)src;
            } else {
                const uint2 b = *(const uint2 *)src;
                seg[q].x = (b.x & 0xFF) | ((b.x & 0xFF00) << 8), seg[q].y = ((b.x >> 16) & 0xFF) | ((b.x >> 8) & 0xFF0000);
                seg[q].z = (b.y & 0xFF) | ((b.y & 0xFF00) << 8), seg[q].w = ((b.y >> 16) & 0xFF) | ((b.y >> 8) & 0xFF0000);
            }
        } else { // the plane's last segment (chroma widths of 4 mod 8): edge-replicated past W
            uint32_t *o = &seg[q].x;
#pragma unroll
            for (int j = 0; j < 4; j++)
                o[j] = (uint32_t)(uint16_t)src[min(2 * j, a.W - 1 - x)] |
                       ((uint32_t)(uint16_t)src[min(2 * j + 1, a.W - 1 - x)] << 16);
        }
    }
    constexpr int IB = (VR * 8 + NTHR - 1) / NTHR; // apron: columns -3..-1 and w..w+4 of each row
    uint16_t      ab[IB];
#pragma unroll
    for (int q = 0; q < IB; q++) {
        const int i = threadIdx.x + q * NTHR, r = (i >> 3) - 3, j = i & 7, cc = j < 3 ? j - 3 : w + j - 3;
        ab[q] = r < h + 4 ? (uint16_t)row_of(r)[min(max(x0 + cc, 0), a.W - 1)] : 0;
    }
#pragma unroll
    for (int q = 0; q < IT; q++) {
        const int i = threadIdx.x + q * NTHR, r = (i >> lseg) - 3, sg = i & ((1 << lseg) - 1);
        if (r < h + 4 && sg < segs) *(uint4 *)(v + (r + 3) * VS + VC0 + 8 * sg) = seg[q];
    }
#pragma unroll
    for (int q = 0; q < IB; q++) {
        const int i = threadIdx.x + q * NTHR, r = (i >> 3) - 3, j = i & 7, cc = j < 3 ? j - 3 : w + j - 3;
        if (r < h + 4) v[(r + 3) * VS + VC0 + cc] = ab[q];
    }
    __syncthreads();
    const uint16_t *v0 = v + 3 * VS + VC0;
    T              *o0 = out + (size_t)y0 * a.out_stride + x0;
    if (u.type == SVTGPU_RESTORE_WIENER)
        wiener_tile(v0, VS, t, TW, w, h, u.hfilter, u.vfilter, a.bd, o0, (size_t)a.out_stride);
    else
        sgr_tile(v0, VS, AB, w, h, u.ep, u.xqd, a.bd, o0, (size_t)a.out_stride);
}

// ---------------------------------------------------------------------------------------------
// RTCD shim kernels (one small block staged compactly)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR) void wiener_shim_kernel(const uint16_t *in, int is, uint16_t *out, int w, int h,
                                                           const int16_t *taps, int bd, int r0, int r1) {
    __shared__ uint16_t t[(64 + 7) * 64];
    __shared__ int16_t  f[16];
    if (threadIdx.x < 16) f[threadIdx.x] = taps[threadIdx.x];
    __syncthreads();
    // custom rounding (the shim honours the caller's ConvolveParams)
    const int lim = (1 << (bd + 1 + 7 - r0)) - 1;
    for (int i = threadIdx.x; i < (h + 7) * w; i += NTHR) {
        const int       y = i / w - 3, x = i % w;
        const uint16_t *s = in + (y + 3) * is + x; // in holds rows/cols from -3
        int             sum = ((int)s[3] << 7) + (1 << (bd + 6));
        for (int k = 0; k < 8; k++) sum += (int)s[k] * f[k];
        t[(y + 3) * w + x] = (uint16_t)min(max((sum + (1 << (r0 - 1))) >> r0, 0), lim);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < h * w; i += NTHR) {
        const int       y = i / w, x = i % w;
        const uint16_t *c = t + y * w + x;
        int             sum = ((int)c[3 * w] << 7) - (1 << (bd + r1 - 1));
        for (int k = 0; k < 8; k++) sum += (int)c[k * w] * f[8 + k];
        out[y * w + x] = (uint16_t)min(max((sum + (1 << (r1 - 1))) >> r1, 0), (1 << bd) - 1);
    }
}

__global__ __launch_bounds__(NTHR) void sgr_shim_kernel(const uint16_t *in, int is, int w, int h, int eps, int bd,
                                                        int32_t x0q, int32_t x1q, int mode, int32_t *flt0,
                                                        int32_t *flt1, uint16_t *out) {
    __shared__ uint16_t v[70 * 70];
    __shared__ int      AB[2][66 * 66];
    for (int i = threadIdx.x; i < (h + 6) * (w + 6); i += NTHR) v[(i / (w + 6)) * 70 + i % (w + 6)] = in[(i / (w + 6)) * is + i % (w + 6)];
    __syncthreads();
    const uint16_t *v0 = v + 3 * 70 + 3;
    const int       bw = w + 2;
    if (mode == 0) { // flt0 / flt1 (svt_av1_selfguided_restoration)
        for (int pass = 0; pass < 2; pass++) {
            const int r = c_sgr_r[eps][pass];
            if (!r) continue;
            for (int i = threadIdx.x; i < (h + 2) * bw; i += NTHR) {
                const int y = i / bw - 1, x = i % bw - 1;
                if (r == 2 && !(y & 1)) continue;
                sgr_ab(v0, 70, y, x, r, c_sgr_s[eps][pass], bd, &AB[0][i], &AB[1][i]);
            }
            __syncthreads();
            for (int i = threadIdx.x; i < w * h; i += NTHR) {
                const int  y = i / w, x = i % w;
                const int *a = AB[0] + (y + 1) * bw + x + 1, *b = AB[1] + (y + 1) * bw + x + 1;
                int        aa, bb, nb;
                if (r == 1) {
                    aa = (a[0] + a[-1] + a[1] + a[-bw] + a[bw]) * 4 + (a[-bw - 1] + a[bw - 1] + a[-bw + 1] + a[bw + 1]) * 3;
                    bb = (b[0] + b[-1] + b[1] + b[-bw] + b[bw]) * 4 + (b[-bw - 1] + b[bw - 1] + b[-bw + 1] + b[bw + 1]) * 3;
                    nb = 5;
                } else if (!(y & 1)) {
                    aa = (a[-bw] + a[bw]) * 6 + (a[-bw - 1] + a[bw - 1] + a[-bw + 1] + a[bw + 1]) * 5;
                    bb = (b[-bw] + b[bw]) * 6 + (b[-bw - 1] + b[bw - 1] + b[-bw + 1] + b[bw + 1]) * 5;
                    nb = 5;
                } else {
                    aa = a[0] * 6 + (a[-1] + a[1]) * 5;
                    bb = b[0] * 6 + (b[-1] + b[1]) * 5;
                    nb = 4;
                }
                const int sh = 8 + nb - 4;
                (pass ? flt1 : flt0)[i] = (aa * (int)v0[y * 70 + x] + bb + (1 << (sh - 1))) >> sh;
            }
            __syncthreads();
        }
    } else {
        const int32_t xqd[2] = {x0q, x1q};
        sgr_tile(v0, 70, (uint32_t *)AB[0], w, h, eps, xqd, bd, out, (size_t)w);
    }
}

} // namespace

// =============================================================================================
// host
// =============================================================================================

namespace {
int count_units(int size, int extent) { return std::max((extent + (size >> 1)) / size, 1); }
} // namespace

extern "C" int svtgpu_lr_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, const int32_t unit_size[3],
                                      SvtGpuLrState **out) {
    if (!ctx || !out || !unit_size || width < 8 || height < 8) return SVTGPU_ERR_INVALID_ARG;
    for (int p = 0; p < 3; p++) {
        const int u = unit_size[p], minu = p ? 32 : 64;
        if (u < minu || u > 256 || (u & (u - 1))) return SVTGPU_ERR_INVALID_ARG;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    SvtGpuLrState *s = new SvtGpuLrState();
    s->ctx           = ctx;
    s->width         = width;
    s->height        = height;
    hipError_t e     = hipSuccess;
    size_t     nu    = 0;
    for (int p = 0; p < 3; p++) {
        const int pw = lr_plane_w(s, p), ph = lr_plane_h(s, p);
        s->unit_size[p] = unit_size[p];
        s->hunits[p]    = count_units(unit_size[p], pw);
        s->vunits[p]    = count_units(unit_size[p], ph);
        s->tile_units[p][0] = s->tile_units[p][1] = 0, s->tile_units[p][2] = s->hunits[p], s->tile_units[p][3] = s->vunits[p];
        s->tile_out[p][0] = s->tile_out[p][1] = 0, s->tile_out[p][2] = pw, s->tile_out[p][3] = ph;
        nu += (size_t)s->hunits[p] * s->vunits[p];
    }
    e = hipMalloc(&s->d_units[0], sizeof(SvtGpuRestUnit) * nu);
    if (e == hipSuccess) e = hipMemset(s->d_units[0], 0, sizeof(SvtGpuRestUnit) * nu);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr); // null-stream memset done before the caller's streams run
    if (e != hipSuccess) s->d_units[0] = nullptr;
    for (int p = 1; p < 3 && s->d_units[0]; p++) s->d_units[p] = s->d_units[p - 1] + s->hunits[p - 1] * s->vunits[p - 1];
    static const bool lazy_wst = [] { // SVTGPU_LR_WST_LAZY=1: the Wiener stream made by the first search (A/B)
        const char *v = std::getenv("SVTGPU_LR_WST_LAZY");
        return v && v[0] == '1';
    }();
    if (e == hipSuccess && !lazy_wst && lr_make_wiener_stream(s) != SVTGPU_OK) e = hipErrorOutOfMemory;
    if (e != hipSuccess) {
        svtgpu_lr_state_destroy(s);
        svtgpu_set_last_hip_error(e, "lr state alloc", __FILE__, __LINE__);
        return e == hipErrorOutOfMemory ? SVTGPU_ERR_OOM : SVTGPU_ERR_HIP;
    }
    *out = s;
    return SVTGPU_OK;
}

extern "C" void svtgpu_lr_state_destroy(SvtGpuLrState *s) {
    if (!s) return;
    (void)hipFree(s->d_units[0]);
    (void)hipFree(s->d_flt);
    (void)hipFree(s->d_work);
    if (s->d_qarena) (void)hipFree(s->d_qarena);
    if (s->d_sxarena) (void)hipFree(s->d_sxarena);
    if (s->pin_free) (void)hipEventSynchronize(s->pin_free), (void)hipEventDestroy(s->pin_free);
    if (s->wst) (void)hipStreamSynchronize(s->wst), (void)hipStreamDestroy(s->wst);
    if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
    if (s->ev_join) (void)hipEventDestroy(s->ev_join);
    if (s->h_pin) (void)hipHostFree(s->h_pin);
    if (s->h_fout) (void)hipHostFree(s->h_fout);
    lr_profiler_destroy(s->prof);
    delete s;
}

extern "C" int svtgpu_lr_units(const SvtGpuLrState *s, int32_t plane, int32_t *hunits, int32_t *vunits) {
    if (!s || plane < 0 || plane > 2) return SVTGPU_ERR_INVALID_ARG;
    if (hunits) *hunits = s->hunits[plane];
    if (vunits) *vunits = s->vunits[plane];
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_set_units(SvtGpuLrState *s, int32_t plane, const SvtGpuRestUnit *units, void *stream) {
    if (!s || !units || plane < 0 || plane > 2) return SVTGPU_ERR_INVALID_ARG;
    const int n = s->hunits[plane] * s->vunits[plane];
    for (int i = 0; i < n; i++) { // the kernels index tables with these fields
        const SvtGpuRestUnit &u = units[i];
        if (u.type < 0 || u.type > 2 || (u.type == SVTGPU_RESTORE_SGRPROJ && (u.ep < 0 || u.ep > 15)))
            return SVTGPU_ERR_INVALID_ARG;
    }
    hipStream_t st = pick_stream(s->ctx, stream);
    HIP_TRY(hipMemcpyAsync(s->d_units[plane], units, sizeof(SvtGpuRestUnit) * n, hipMemcpyHostToDevice, st));
    svtgpu_count_xfer(0, sizeof(SvtGpuRestUnit) * n);
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

extern "C" int svtgpu_lr_apply_frame(SvtGpuLrState *s, const SvtGpuFrame *deblocked, const SvtGpuFrame *cdef_out,
                                     SvtGpuFrame *out, const int32_t frame_type[3], void *stream) {
    auto ok = [&](const SvtGpuFrame *f) {
        return lr_frame_fits(s, f) && f->bit_depth == cdef_out->bit_depth;
    };
    if (!s || !cdef_out || !ok(cdef_out) || !ok(deblocked) || !ok(out) || out == cdef_out || out == deblocked)
        return SVTGPU_ERR_INVALID_ARG;
    if (cdef_out->bit_depth != 8 && cdef_out->bit_depth != 10) return SVTGPU_ERR_UNSUPPORTED;
    hipStream_t  st  = pick_stream(s->ctx, stream);
    const size_t bps = cdef_out->bytes_per_sample;
    LrApplyArgs  L;
    L.nplanes = 0;
    int nblk  = 0;
    for (int p = 0; p < 3; p++) {
        const int32_t *r = s->tile_out[p]; // the samples written (the whole plane unless tiled over GPUs)
        // a crop size below the coded size: the samples right of / below the restored area keep the CDEF output
        // (the reference filters crop_widths x crop_heights only, EbRestoration.c:1216-1217)
        const int pw = lr_plane_w(s, p), ph = lr_plane_h(s, p);
        if (r[2] == pw && pw < cdef_out->pw[p])
            HIP_TRY(hipMemcpy2DAsync((uint8_t *)out->plane[p] + ((size_t)r[1] * out->stride[p] + pw) * bps,
                                     out->stride[p] * bps,
                                     (const uint8_t *)cdef_out->plane[p] + ((size_t)r[1] * cdef_out->stride[p] + pw) * bps,
                                     cdef_out->stride[p] * bps, (cdef_out->pw[p] - pw) * bps, r[3] - r[1],
                                     hipMemcpyDeviceToDevice, st));
        if (r[3] == ph && ph < cdef_out->ph[p])
            HIP_TRY(hipMemcpy2DAsync((uint8_t *)out->plane[p] + ((size_t)ph * out->stride[p] + r[0]) * bps,
                                     out->stride[p] * bps,
                                     (const uint8_t *)cdef_out->plane[p] + ((size_t)ph * cdef_out->stride[p] + r[0]) * bps,
                                     cdef_out->stride[p] * bps,
                                     ((r[2] == pw ? cdef_out->pw[p] : r[2]) - r[0]) * bps, cdef_out->ph[p] - ph,
                                     hipMemcpyDeviceToDevice, st));
        // frame_type == nullptr: the units the last search left on the device (an asynchronous search's device finish:
        // a plane whose frame type is NONE holds NONE units, which the kernel copies)
        if (frame_type && frame_type[p] == SVTGPU_RESTORE_NONE) {
            const size_t io = ((size_t)r[1] * cdef_out->stride[p] + r[0]) * bps, oo = ((size_t)r[1] * out->stride[p] + r[0]) * bps;
            HIP_TRY(hipMemcpy2DAsync((uint8_t *)out->plane[p] + oo, out->stride[p] * bps,
                                     (const uint8_t *)cdef_out->plane[p] + io, cdef_out->stride[p] * bps,
                                     (r[2] - r[0]) * bps, r[3] - r[1], hipMemcpyDeviceToDevice, st));
            continue;
        }
        LrPlaneArgs &a = L.pl[L.nplanes];
        a.dlf         = deblocked->plane[p];
        a.cdef        = cdef_out->plane[p];
        a.out         = out->plane[p];
        a.dlf_stride  = deblocked->stride[p];
        a.cdef_stride = cdef_out->stride[p];
        a.out_stride  = out->stride[p];
        a.W           = pw;
        a.H           = ph;
        a.ss          = p > 0;
        a.unit_size   = s->unit_size[p];
        a.hunits      = s->hunits[p];
        a.vunits      = s->vunits[p];
        a.bd          = cdef_out->bit_depth;
        a.units       = s->d_units[p];
        const int S = 64 >> a.ss, off = 8 >> a.ss, cw = 64 >> a.ss;
        a.nchunks     = (a.W + cw - 1) / cw;
        // the rect is a union of whole (stripe, chunk) tiles (svtgpu_lr_set_tile checks)
        a.k0 = (r[1] + off) / S, a.c0 = r[0] / cw, a.nc = (r[2] + cw - 1) / cw - a.c0;
        const int nk = (r[3] + off + S - 1) / S - a.k0;
        a.count = nk * a.nc;
        nblk += (a.count + 7) & ~7;
        L.end[L.nplanes++] = nblk;
    }
    if (!nblk) return SVTGPU_OK;
    if (bps == 2)
        hipLaunchKernelGGL(lr_apply_kernel<uint16_t>, dim3(nblk), dim3(NTHR), 0, st, L);
    else
        hipLaunchKernelGGL(lr_apply_kernel<uint8_t>, dim3(nblk), dim3(NTHR), 0, st, L);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

// ---------------------------------------------------------------------------------------------
// shims
// ---------------------------------------------------------------------------------------------
namespace {
struct ShimBuf {
    void  *p = nullptr;
    size_t n = 0;
    void  *get(size_t b) {
        if (b > n) {
            if (p) (void)hipFree(p);
            HIP_OR_DIE(hipMalloc(&p, b));
            n = b;
        }
        return p;
    }
};
thread_local ShimBuf g_lr_buf;

const int kHostSgrR[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                              {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};
inline bool c_host_r0(int eps) { return kHostSgrR[eps][0] > 0; }
inline bool c_host_r1(int eps) { return kHostSgrR[eps][1] > 0; }

template <typename T>
void wiener_shim(const T *src, ptrdiff_t ss, T *dst, ptrdiff_t ds, const int16_t *fx, const int16_t *fy, int w, int h,
                 int r0, int r1, int bd) {
    if (w <= 0 || h <= 0 || w > 64 || h > 64) svtgpu_fatal("wiener shim: block larger than 64x64");
    const int             is = w + 8;
    std::vector<uint16_t> in((size_t)(h + 8) * is);
    for (int y = -3; y < h + 5; y++)
        for (int x = -3; x < w + 5; x++) in[(size_t)(y + 3) * is + x + 3] = src[y * ss + x];
    int16_t taps[16];
    std::memcpy(taps, fx, 16);
    std::memcpy(taps + 8, fy, 16);
    uint8_t  *d    = (uint8_t *)g_lr_buf.get(in.size() * 2 + (size_t)w * h * 2 + 64);
    uint16_t *di   = (uint16_t *)d, *dout = (uint16_t *)(d + in.size() * 2);
    int16_t  *dt   = (int16_t *)(d + in.size() * 2 + (size_t)w * h * 2);
    hipStream_t st = svtgpu_shim_stream();
    HIP_OR_DIE(hipMemcpyAsync(di, in.data(), in.size() * 2, hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(dt, taps, 32, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(wiener_shim_kernel, dim3(1), dim3(NTHR), 0, st, di, is, dout, w, h, dt, bd, r0, r1);
    HIP_OR_DIE(hipGetLastError());
    std::vector<uint16_t> res((size_t)w * h);
    HIP_OR_DIE(hipMemcpyAsync(res.data(), dout, res.size() * 2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) dst[y * ds + x] = (T)res[(size_t)y * w + x];
}

template <typename T>
void sgr_shim(const T *src, int stride, int w, int h, int eps, const int32_t *xqd, int bd, int mode, int32_t *flt0,
              int32_t *flt1, int fstride, T *dst, int dstride) {
    if (w <= 0 || h <= 0 || w > 64 || h > 64 || eps < 0 || eps > 15) svtgpu_fatal("sgr shim: bad block");
    const int             is = w + 6;
    std::vector<uint16_t> in((size_t)(h + 6) * is);
    for (int y = -3; y < h + 3; y++)
        for (int x = -3; x < w + 3; x++) in[(size_t)(y + 3) * is + x + 3] = src[y * stride + x];
    const size_t nb = in.size() * 2, no = (size_t)w * h;
    uint8_t     *d  = (uint8_t *)g_lr_buf.get(nb + no * 10 + 64);
    uint16_t    *di = (uint16_t *)d;
    int32_t     *f0 = (int32_t *)(d + ((nb + 15) & ~15)), *f1 = f0 + no;
    uint16_t    *dout = (uint16_t *)(f1 + no);
    hipStream_t  st   = svtgpu_shim_stream();
    HIP_OR_DIE(hipMemcpyAsync(di, in.data(), nb, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(sgr_shim_kernel, dim3(1), dim3(NTHR), 0, st, di, is, w, h, eps, bd, xqd ? xqd[0] : 0,
                       xqd ? xqd[1] : 0, mode, f0, f1, dout);
    HIP_OR_DIE(hipGetLastError());
    std::vector<int32_t>  r0(no), r1(no);
    std::vector<uint16_t> ro(no);
    if (mode == 0) {
        HIP_OR_DIE(hipMemcpyAsync(r0.data(), f0, no * 4, hipMemcpyDeviceToHost, st));
        HIP_OR_DIE(hipMemcpyAsync(r1.data(), f1, no * 4, hipMemcpyDeviceToHost, st));
    } else
        HIP_OR_DIE(hipMemcpyAsync(ro.data(), dout, no * 2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            if (mode == 0) {
                // the reference writes only the filters its radii enable
                if (flt0 && c_host_r0(eps)) flt0[y * fstride + x] = r0[(size_t)y * w + x];
                if (flt1 && c_host_r1(eps)) flt1[y * fstride + x] = r1[(size_t)y * w + x];
            } else
                dst[y * dstride + x] = (T)ro[(size_t)y * w + x];
        }
}
} // namespace

extern "C" void svtgpu_av1_wiener_convolve_add_src(const uint8_t *src, ptrdiff_t src_stride, uint8_t *dst,
                                                   ptrdiff_t dst_stride, const int16_t *filter_x,
                                                   const int16_t *filter_y, int32_t w, int32_t h,
                                                   const SvtGpuConvolveParams *conv_params) {
    wiener_shim<uint8_t>(src, src_stride, dst, dst_stride, filter_x, filter_y, w, h, conv_params->round_0,
                         conv_params->round_1, 8);
}

extern "C" void svtgpu_av1_highbd_wiener_convolve_add_src(const uint8_t *src, ptrdiff_t src_stride, uint8_t *dst,
                                                          ptrdiff_t dst_stride, const int16_t *filter_x,
                                                          const int16_t *filter_y, int32_t w, int32_t h,
                                                          const SvtGpuConvolveParams *conv_params, int32_t bd) {
    wiener_shim<uint16_t>((const uint16_t *)((uintptr_t)src << 1), src_stride, (uint16_t *)((uintptr_t)dst << 1),
                          dst_stride, filter_x, filter_y, w, h, conv_params->round_0, conv_params->round_1, bd);
}

extern "C" void svtgpu_av1_selfguided_restoration(const uint8_t *dgd8, int32_t width, int32_t height,
                                                  int32_t dgd_stride, int32_t *flt0, int32_t *flt1, int32_t flt_stride,
                                                  int32_t sgr_params_idx, int32_t bit_depth, int32_t highbd) {
    if (highbd)
        sgr_shim<uint16_t>((const uint16_t *)((uintptr_t)dgd8 << 1), dgd_stride, width, height, sgr_params_idx,
                           nullptr, bit_depth, 0, flt0, flt1, flt_stride, nullptr, 0);
    else
        sgr_shim<uint8_t>(dgd8, dgd_stride, width, height, sgr_params_idx, nullptr, bit_depth, 0, flt0, flt1,
                          flt_stride, nullptr, 0);
}

extern "C" void svtgpu_apply_selfguided_restoration(const uint8_t *dat8, int32_t width, int32_t height, int32_t stride,
                                                    int32_t eps, const int32_t *xqd, uint8_t *dst8, int32_t dst_stride,
                                                    int32_t *tmpbuf, int32_t bit_depth, int32_t highbd) {
    (void)tmpbuf;
    if (highbd)
        sgr_shim<uint16_t>((const uint16_t *)((uintptr_t)dat8 << 1), stride, width, height, eps, xqd, bit_depth, 1,
                           nullptr, nullptr, 0, (uint16_t *)((uintptr_t)dst8 << 1), dst_stride);
    else
        sgr_shim<uint8_t>(dat8, stride, width, height, eps, xqd, bit_depth, 1, nullptr, nullptr, 0, dst8, dst_stride);
}
