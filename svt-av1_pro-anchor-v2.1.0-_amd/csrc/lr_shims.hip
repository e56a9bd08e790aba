// lr_shims.hip — RTCD-compatible per-unit shims of the loop-restoration search (host pointers, synchronous).
//
// The frame-level search (lr_search.hip) keeps its statistics, filter planes and projections on the device; these
// entry points exist so the reference's own search loop (EbRestorationPick.c) and its unit tests can run on the
// device through the function pointers they already call:
//   svtgpu_av1_compute_stats(_highbd)      ≙ svt_av1_compute_stats(_highbd)   (aom_dsp_rtcd.h:66-68, C :671 / :708):
//                                            the frame search's MFMA kernel (8/10-bit), a VALU kernel (12-bit)
//   svtgpu_av1_lowbd/highbd_pixel_proj_error ≙ svt_av1_*_pixel_proj_error     (aom_dsp_rtcd.h:79-81, C :167 / :232)
//   svtgpu_get_proj_subspace               ≙ svt_get_proj_subspace            (aom_dsp_rtcd.h:212, C :560)
// Every sum is integer on the device; get_proj_subspace's double sums are sums of integers below 2^53 in the
// reference, hence exact, so the int64 totals converted to double reproduce them, and the 2x2 solve that follows
// runs on the host in the reference's order (-ffp-contract=off).
#include <cmath>
#include <cstring>
#include <vector>

#include "svtgpu_internal.h"

namespace {
constexpr int kRstBits = 4, kPrjBits = 7; // SGRPROJ_RST_BITS, SGRPROJ_PRJ_BITS (EbRestoration.h:94-96)

struct DevBuf { // per-thread grow-only device staging
    void  *p   = nullptr;
    size_t cap = 0;
    void  *get(size_t n) {
        if (n > cap) {
            if (p) (void)hipFree(p);
            HIP_OR_DIE(hipMalloc(&p, n));
            cap = n;
        }
        return p;
    }
};
thread_local DevBuf g_lr_scratch;

inline const uint16_t *short_ptr(const uint8_t *p) { return (const uint16_t *)((uintptr_t)p << 1); }

template <typename T>
__global__ __launch_bounds__(256) void lr_sum_kernel(const T *a, int stride, int w, int h, unsigned long long *out) {
    unsigned long long s = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < w * h; i += gridDim.x * 256) s += a[(i / w) * stride + i % w];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

// one lane per M entry (q < win2) and per H entry (win2 + p * win2 + q); window sample q sits at column offset
// q / win - half, row offset q % win - half (the reference's y[] order, EbRestorationPick.c:684-690)
template <typename T, typename Acc>
__global__ __launch_bounds__(256) void lr_stats_kernel(int win, const T *dgd, int ds, const T *src, int ss, int w, int h,
                                                       const unsigned long long *sum, int64_t *M, int64_t *H, int div) {
    const int win2 = win * win, e = blockIdx.x * 256 + threadIdx.x, half = win >> 1;
    if (e >= win2 + win2 * win2) return;
    const Acc avg = (Acc)(T)(*sum / (unsigned long long)(w * h)); // find_average(_highbd): truncating, then narrowed
    const bool is_m = e < win2;
    const int  p = is_m ? e : (e - win2) / win2, q = is_m ? e : (e - win2) % win2;
    const int  pc = p / win - half, pr = p % win - half, qc = q / win - half, qr = q % win - half;
    int64_t    acc = 0;
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            const Acc yp = (Acc)dgd[(i + pr) * ds + j + pc] - avg;
            const Acc o  = is_m ? (Acc)src[i * ss + j] - avg : (Acc)dgd[(i + qr) * ds + j + qc] - avg;
            acc += (int64_t)yp * o;
        }
    acc /= div; // the highbd divider (1 for 8-bit): the reference divides after accumulating
    if (is_m)
        M[p] = acc;
    else
        H[p * win2 + q] = acc;
}

template <typename T>
void compute_stats(int32_t win, const T *dgd, const T *src, int32_t h_start, int32_t h_end, int32_t v_start,
                   int32_t v_end, int32_t dgd_stride, int32_t src_stride, int64_t *M, int64_t *H, int div) {
    const int half = win >> 1, w = h_end - h_start, h = v_end - v_start, win2 = win * win;
    const int dw = w + 2 * half, dh = h + 2 * half;
    std::vector<T> hd((size_t)dw * dh), hs((size_t)w * h);
    for (int r = 0; r < dh; r++)
        memcpy(&hd[(size_t)r * dw], dgd + (long)(v_start - half + r) * dgd_stride + h_start - half, sizeof(T) * dw);
    for (int r = 0; r < h; r++) memcpy(&hs[(size_t)r * w], src + (long)(v_start + r) * src_stride + h_start, sizeof(T) * w);
    const size_t od = 0, os = (hd.size() * sizeof(T) + 255) & ~(size_t)255, osum = os + ((hs.size() * sizeof(T) + 255) & ~(size_t)255);
    const size_t om = osum + 256, oh = om + 8 * 64;
    char        *d = (char *)g_lr_scratch.get(oh + (size_t)8 * win2 * win2);
    hipStream_t  st = svtgpu_shim_stream();
    HIP_OR_DIE(hipMemcpyAsync(d + od, hd.data(), hd.size() * sizeof(T), hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + os, hs.data(), hs.size() * sizeof(T), hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemsetAsync(d + osum, 0, 8, st));
    const T *dd = (const T *)(d + od) + (size_t)half * dw + half;
    hipLaunchKernelGGL(lr_sum_kernel<T>, dim3(64), dim3(256), 0, st, dd, dw, w, h, (unsigned long long *)(d + osum));
    const int n = win2 + win2 * win2;
    if (sizeof(T) == 1)
        hipLaunchKernelGGL((lr_stats_kernel<T, int16_t>), dim3((n + 255) / 256), dim3(256), 0, st, win, dd, dw,
                           (const T *)(d + os), w, w, h, (const unsigned long long *)(d + osum), (int64_t *)(d + om),
                           (int64_t *)(d + oh), div);
    else
        hipLaunchKernelGGL((lr_stats_kernel<T, int32_t>), dim3((n + 255) / 256), dim3(256), 0, st, win, dd, dw,
                           (const T *)(d + os), w, w, h, (const unsigned long long *)(d + osum), (int64_t *)(d + om),
                           (int64_t *)(d + oh), div);
    HIP_OR_DIE(hipGetLastError());
    HIP_OR_DIE(hipMemcpyAsync(M, d + om, 8 * (size_t)win2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipMemcpyAsync(H, d + oh, 8 * (size_t)win2 * win2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
}

// ---- projection error / subspace: per-sample terms, integer reductions ----
// mode: 0 both filters, 1 flt0 only, 2 flt1 only, 3 none (r[0] / r[1] of the ep's SgrParamsType)
template <typename T, bool HBD>
__global__ __launch_bounds__(256) void proj_err_shim_kernel(const T *src, const T *dat, const int32_t *f0,
                                                            const int32_t *f1, int w, int h, int xq0, int xq1,
                                                            int mode, unsigned long long *out) {
    unsigned long long acc = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < w * h; i += gridDim.x * 256) {
        const int32_t d = dat[i], s = src[i], u = d << kRstBits;
        int32_t       e;
        if (mode == 3) {
            e = d - s;
        } else {
            int32_t v = HBD ? (1 << (kRstBits + kPrjBits - 1)) : (u << kPrjBits);
            if (mode != 2) v += xq0 * (f0[i] - u);
            if (mode != 1) v += xq1 * (f1[i] - u);
            // lowbd: ROUND_POWER_OF_TWO(v, 11) - s (:181); highbd: (v >> 11) + d - s with the half pre-added (:254)
            e = HBD ? (v >> (kRstBits + kPrjBits)) + d - s : ((v + (1 << (kRstBits + kPrjBits - 1))) >> (kRstBits + kPrjBits)) - s;
        }
        acc += (unsigned long long)(long long)(e * e);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

template <typename T>
__global__ __launch_bounds__(256) void proj_sub_shim_kernel(const T *src, const T *dat, const int32_t *f0,
                                                            const int32_t *f1, int w, int h, int use0, int use1,
                                                            unsigned long long *out) {
    long long a[5] = {0, 0, 0, 0, 0}; // H00, H11, H01, C0, C1
    for (int i = blockIdx.x * 256 + threadIdx.x; i < w * h; i += gridDim.x * 256) {
        const long long u  = (long long)dat[i] << kRstBits;
        const long long s  = ((long long)src[i] << kRstBits) - u;
        const long long g1 = use0 ? f0[i] - u : 0, g2 = use1 ? f1[i] - u : 0;
        a[0] += g1 * g1, a[1] += g2 * g2, a[2] += g1 * g2, a[3] += g1 * s, a[4] += g2 * s;
    }
    for (int k = 0; k < 5; k++) {
        for (int o = 32; o > 0; o >>= 1) a[k] += __shfl_down(a[k], o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&out[k], (unsigned long long)a[k]);
    }
}

template <typename T>
struct ProjStage {
    const T       *src, *dat;
    const int32_t *f0, *f1;
    char          *d;
};
template <typename T>
ProjStage<T> stage_proj(const T *src, int sst, const T *dat, int dst, const int32_t *flt0, int f0s, const int32_t *flt1,
                        int f1s, int w, int h, bool use0, bool use1, hipStream_t st) {
    const size_t npx = (size_t)w * h, ot = (npx * sizeof(T) + 255) & ~(size_t)255, of = (npx * 4 + 255) & ~(size_t)255;
    char        *d = (char *)g_lr_scratch.get(2 * ot + 2 * of + 256);
    std::vector<char> buf(std::max(ot, of));
    auto put = [&](size_t off, const void *base, int stride, size_t es) {
        for (int r = 0; r < h; r++) memcpy(buf.data() + (size_t)r * w * es, (const char *)base + (size_t)r * stride * es, (size_t)w * es);
        HIP_OR_DIE(hipMemcpyAsync(d + off, buf.data(), npx * es, hipMemcpyHostToDevice, st));
        HIP_OR_DIE(hipStreamSynchronize(st)); // buf is reused
    };
    put(0, src, sst, sizeof(T));
    put(ot, dat, dst, sizeof(T));
    if (use0) put(2 * ot, flt0, f0s, 4);
    if (use1) put(2 * ot + of, flt1, f1s, 4);
    HIP_OR_DIE(hipMemsetAsync(d + 2 * ot + 2 * of, 0, 64, st));
    return {(const T *)d, (const T *)(d + ot), (const int32_t *)(d + 2 * ot), (const int32_t *)(d + 2 * ot + of),
            d + 2 * ot + 2 * of};
}

template <typename T, bool HBD>
int64_t pixel_proj_error(const T *src, int32_t width, int32_t height, int32_t src_stride, const T *dat,
                         int32_t dat_stride, const int32_t *flt0, int32_t flt0_stride, const int32_t *flt1,
                         int32_t flt1_stride, const int32_t xq[2], const SVTGPU_SGR_PARAMS_T *params) {
    const bool  use0 = params->r[0] > 0, use1 = params->r[1] > 0;
    const int   mode = use0 && use1 ? 0 : use0 ? 1 : use1 ? 2 : 3;
    hipStream_t st   = svtgpu_shim_stream();
    auto        S    = stage_proj<T>(src, src_stride, dat, dat_stride, flt0, flt0_stride, flt1, flt1_stride, width,
                                     height, use0, use1, st);
    hipLaunchKernelGGL((proj_err_shim_kernel<T, HBD>), dim3(32), dim3(256), 0, st, S.src, S.dat, S.f0, S.f1, width,
                       height, xq[0], xq[1], mode, (unsigned long long *)S.d);
    HIP_OR_DIE(hipGetLastError());
    unsigned long long r;
    HIP_OR_DIE(hipMemcpyAsync(&r, S.d, 8, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    return (int64_t)r;
}
} // namespace

// 8- and 10-bit: the frame search's MFMA statistics kernel (svtgpu_stats_unit_mfma*, lr_search.hip), so the reference's
// own compute_stats vectors check it directly; 12-bit samples overflow its i32 wave fold and take the VALU kernel above
extern "C" void svtgpu_av1_compute_stats(int32_t wiener_win, const uint8_t *dgd8, const uint8_t *src8, int32_t h_start,
                                         int32_t h_end, int32_t v_start, int32_t v_end, int32_t dgd_stride,
                                         int32_t src_stride, int64_t *M, int64_t *H) {
    if (svtgpu_stats_unit_mfma8(wiener_win, dgd8, src8, h_start, h_end, v_start, v_end, dgd_stride, src_stride, M, H))
        svtgpu_fatal("svtgpu_av1_compute_stats");
}

extern "C" void svtgpu_av1_compute_stats_highbd(int32_t wiener_win, const uint8_t *dgd8, const uint8_t *src8,
                                                int32_t h_start, int32_t h_end, int32_t v_start, int32_t v_end,
                                                int32_t dgd_stride, int32_t src_stride, int64_t *M, int64_t *H,
                                                int32_t bit_depth) {
    const int div = bit_depth == 12 ? 16 : bit_depth == 10 ? 4 : 1; // EbRestorationPick.c:716-720
    if (bit_depth <= 10) {
        if (svtgpu_stats_unit_mfma16(wiener_win, short_ptr(dgd8), short_ptr(src8), h_start, h_end, v_start, v_end,
                                     dgd_stride, src_stride, M, H, div))
            svtgpu_fatal("svtgpu_av1_compute_stats_highbd");
        return;
    }
    compute_stats<uint16_t>(wiener_win, short_ptr(dgd8), short_ptr(src8), h_start, h_end, v_start, v_end, dgd_stride,
                            src_stride, M, H, div);
}

extern "C" int64_t svtgpu_av1_lowbd_pixel_proj_error(const uint8_t *src8, int32_t width, int32_t height,
                                                     int32_t src_stride, const uint8_t *dat8, int32_t dat_stride,
                                                     int32_t *flt0, int32_t flt0_stride, int32_t *flt1,
                                                     int32_t flt1_stride, int32_t xq[2],
                                                     const SVTGPU_SGR_PARAMS_T *params) {
    return pixel_proj_error<uint8_t, false>(src8, width, height, src_stride, dat8, dat_stride, flt0, flt0_stride, flt1,
                                            flt1_stride, xq, params);
}

extern "C" int64_t svtgpu_av1_highbd_pixel_proj_error(const uint8_t *src8, int32_t width, int32_t height,
                                                      int32_t src_stride, const uint8_t *dat8, int32_t dat_stride,
                                                      int32_t *flt0, int32_t flt0_stride, int32_t *flt1,
                                                      int32_t flt1_stride, int32_t xq[2],
                                                      const SVTGPU_SGR_PARAMS_T *params) {
    return pixel_proj_error<uint16_t, true>(short_ptr(src8), width, height, src_stride, short_ptr(dat8), dat_stride,
                                            flt0, flt0_stride, flt1, flt1_stride, xq, params);
}

extern "C" void svtgpu_get_proj_subspace(const uint8_t *src8, int width, int height, int src_stride,
                                         const uint8_t *dat8, int dat_stride, int use_highbitdepth, int32_t *flt0,
                                         int flt0_stride, int32_t *flt1, int flt1_stride, int *xq,
                                         const SVTGPU_SGR_PARAMS_T *params) {
    const bool         use0 = params->r[0] > 0, use1 = params->r[1] > 0;
    hipStream_t        st   = svtgpu_shim_stream();
    unsigned long long r[5];
    if (use_highbitdepth) {
        auto S = stage_proj<uint16_t>(short_ptr(src8), src_stride, short_ptr(dat8), dat_stride, flt0, flt0_stride, flt1,
                                      flt1_stride, width, height, use0, use1, st);
        hipLaunchKernelGGL(proj_sub_shim_kernel<uint16_t>, dim3(32), dim3(256), 0, st, S.src, S.dat, S.f0, S.f1, width,
                           height, (int)use0, (int)use1, (unsigned long long *)S.d);
        HIP_OR_DIE(hipMemcpyAsync(r, S.d, sizeof r, hipMemcpyDeviceToHost, st));
    } else {
        auto S = stage_proj<uint8_t>(src8, src_stride, dat8, dat_stride, flt0, flt0_stride, flt1, flt1_stride, width,
                                     height, use0, use1, st);
        hipLaunchKernelGGL(proj_sub_shim_kernel<uint8_t>, dim3(32), dim3(256), 0, st, S.src, S.dat, S.f0, S.f1, width,
                           height, (int)use0, (int)use1, (unsigned long long *)S.d);
        HIP_OR_DIE(hipMemcpyAsync(r, S.d, sizeof r, hipMemcpyDeviceToHost, st));
    }
    HIP_OR_DIE(hipGetLastError());
    HIP_OR_DIE(hipStreamSynchronize(st));
    // EbRestorationPick.c:595-640, in the reference's order
    const double size = (double)(width * height);
    double       H00 = (double)(int64_t)r[0] / size, H11 = (double)(int64_t)r[1] / size, H01 = (double)(int64_t)r[2] / size;
    double       C0 = (double)(int64_t)r[3] / size, C1 = (double)(int64_t)r[4] / size;
    const double H10 = H01;
    xq[0] = xq[1] = 0;
    if (params->r[0] == 0) {
        const double det = H11;
        if (det < 1e-8) return;
        xq[1] = (int32_t)rint(C1 / det * (1 << kPrjBits));
    } else if (params->r[1] == 0) {
        const double det = H00;
        if (det < 1e-8) return;
        xq[0] = (int32_t)rint(C0 / det * (1 << kPrjBits));
    } else {
        const double det = H00 * H11 - H01 * H10;
        if (det < 1e-8) return;
        const double x0 = (H11 * C0 - H01 * C1) / det, x1 = (H00 * C1 - H10 * C0) / det;
        xq[0] = (int32_t)rint(x0 * (1 << kPrjBits));
        xq[1] = (int32_t)rint(x1 * (1 << kPrjBits));
    }
}
