// cdef_block.hip — RTCD-compatible per-block CDEF entry points (unit parity with the reference's
// gtests; see include/svtgpu.h layer 1).  Each call stages its operands to the device, runs one
// small HIP kernel and copies the result back synchronously on the library's default context.
#include <cstring>
#include <vector>

#include "cdef_common.h"

namespace {
struct DevBuf { // grow-only device scratch for the shims (one per thread)
    void  *p = nullptr;
    size_t n = 0;
    void  *get(size_t bytes) {
        if (bytes > n) {
            if (p) (void)hipFree(p);
            HIP_OR_DIE(hipMalloc(&p, bytes));
            n = bytes;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
thread_local DevBuf g_scratch;
} // namespace

// ---------------------------------------------------------------------------------------------
// direction: svt_aom_cdef_find_dir_c (EbCdef.c:150-210), one lane per 8x8 block
// ---------------------------------------------------------------------------------------------
__global__ void cdef_find_dir_kernel(const uint16_t *img, int n, int cs, uint8_t *dir, int32_t *var) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    const uint16_t *p = img + b * 64;
    int line[8][15];
    for (int d = 0; d < 8; d++)
        for (int k = 0; k < 15; k++) line[d][k] = 0;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            const int x = (p[i * 8 + j] >> cs) - 128;
            line[0][i + j] += x;
            line[1][i + j / 2] += x;
            line[2][i] += x;
            line[3][3 + i - j / 2] += x;
            line[4][7 + i - j] += x;
            line[5][3 - i / 2 + j] += x;
            line[6][j] += x;
            line[7][i / 2 + j] += x;
        }
    const int w840[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
    int       cost[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 8; k++) {
        cost[2] += line[2][k] * line[2][k];
        cost[6] += line[6][k] * line[6][k];
    }
    cost[2] *= w840[8];
    cost[6] *= w840[8];
    for (int k = 0; k < 7; k++) {
        cost[0] += (line[0][k] * line[0][k] + line[0][14 - k] * line[0][14 - k]) * w840[k + 1];
        cost[4] += (line[4][k] * line[4][k] + line[4][14 - k] * line[4][14 - k]) * w840[k + 1];
    }
    cost[0] += line[0][7] * line[0][7] * w840[8];
    cost[4] += line[4][7] * line[4][7] * w840[8];
    for (int d = 1; d < 8; d += 2) {
        for (int k = 3; k < 8; k++) cost[d] += line[d][k] * line[d][k];
        cost[d] *= w840[8];
        for (int k = 0; k < 3; k++) cost[d] += (line[d][k] * line[d][k] + line[d][10 - k] * line[d][10 - k]) * w840[2 * k + 2];
    }
    int best = 0, bd = 0;
    for (int d = 0; d < 8; d++)
        if (cost[d] > best) {
            best = cost[d];
            bd   = d;
        }
    dir[b] = (uint8_t)bd;
    var[b] = (best - cost[(bd + 4) & 7]) >> 10;
}

static void find_dir_batch(const uint16_t *const *imgs, int stride, int n, int cs, uint8_t *dirs, int32_t *vars) {
    hipStream_t           st = svtgpu_shim_stream();
    std::vector<uint16_t> h((size_t)n * 64);
    for (int b = 0; b < n; b++)
        for (int i = 0; i < 8; i++) memcpy(&h[(size_t)b * 64 + i * 8], imgs[b] + (size_t)i * stride, 16);
    char *d = (char *)g_scratch.get((size_t)n * (128 + 1 + 4) + 64);
    HIP_OR_DIE(hipMemcpyAsync(d, h.data(), (size_t)n * 128, hipMemcpyHostToDevice, st));
    uint8_t *dd = (uint8_t *)(d + (size_t)n * 128);
    int32_t *dv = (int32_t *)(d + (size_t)n * 128 + ((n + 3) & ~3));
    hipLaunchKernelGGL(cdef_find_dir_kernel, dim3((n + 63) / 64), dim3(64), 0, st, (const uint16_t *)d, n, cs, dd, dv);
    HIP_OR_DIE(hipGetLastError());
    HIP_OR_DIE(hipMemcpyAsync(dirs, dd, n, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipMemcpyAsync(vars, dv, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
}

extern "C" uint8_t svtgpu_cdef_find_dir(const uint16_t *img, int32_t stride, int32_t *var, int32_t coeff_shift) {
    uint8_t d;
    find_dir_batch(&img, stride, 1, coeff_shift, &d, var);
    return d;
}

extern "C" void svtgpu_cdef_find_dir_dual(const uint16_t *img1, const uint16_t *img2, int stride, int32_t *var1,
                                          int32_t *var2, int32_t coeff_shift, uint8_t *out1, uint8_t *out2) {
    const uint16_t *imgs[2] = {img1, img2};
    uint8_t         d[2];
    int32_t         v[2];
    find_dir_batch(imgs, stride, 2, coeff_shift, d, v);
    *out1 = d[0];
    *out2 = d[1];
    *var1 = v[0];
    *var2 = v[1];
}

// ---------------------------------------------------------------------------------------------
// filter: svt_cdef_filter_block_c (EbCdef.c:253-300), one lane per output sample
// ---------------------------------------------------------------------------------------------
__global__ void cdef_filter_block_kernel(const uint16_t *win, int ws, int bh, int bw, int pri, int sec, int dir,
                                         int pdamp, int sdamp, int cs, int ss, uint16_t *out) {
    const int i = threadIdx.x / bw, j = threadIdx.x % bw;
    if (i >= bh || (i % ss)) return;
    const uint16_t *p = win + (i + CDEF_BORDER) * ws + j + CDEF_BORDER;
    out[i * bw + j]   = (uint16_t)cdef_filter_px(p, ws, pri, sec, dir, pdamp, sdamp, cs);
}

extern "C" void svtgpu_cdef_filter_block(uint8_t *dst8, uint16_t *dst16, int32_t dstride, const uint16_t *in,
                                         int32_t pri_strength, int32_t sec_strength, int32_t dir, int32_t pri_damping,
                                         int32_t sec_damping, int32_t bsize, int32_t coeff_shift,
                                         uint8_t subsampling_factor) {
    const int bh = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_4X8) ? 8 : 4;
    const int bw = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_8X4) ? 8 : 4;
    const int ws = bw + 2 * CDEF_BORDER, wh = bh + 2 * CDEF_BORDER;
    const int ss = subsampling_factor ? subsampling_factor : 1;
    std::vector<uint16_t> win((size_t)ws * wh);
    for (int r = 0; r < wh; r++) // exactly the samples the reference reads (rows/cols -2..+1 past the block)
        memcpy(&win[(size_t)r * ws], in + (long)(r - CDEF_BORDER) * 144 - CDEF_BORDER, (size_t)ws * 2);
    hipStream_t st = svtgpu_shim_stream();
    char       *d  = (char *)g_scratch.get(win.size() * 2 + 256);
    uint16_t   *dout = (uint16_t *)(d + ((win.size() * 2 + 15) & ~(size_t)15));
    HIP_OR_DIE(hipMemcpyAsync(d, win.data(), win.size() * 2, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(cdef_filter_block_kernel, dim3(1), dim3(64), 0, st, (const uint16_t *)d, ws, bh, bw, pri_strength,
                       sec_strength, dir, pri_damping, sec_damping, coeff_shift, ss, dout);
    HIP_OR_DIE(hipGetLastError());
    uint16_t out[64];
    HIP_OR_DIE(hipMemcpyAsync(out, dout, 128, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int i = 0; i < bh; i += ss)
        for (int j = 0; j < bw; j++) {
            if (dst8)
                dst8[i * dstride + j] = (uint8_t)out[i * bw + j];
            else
                dst16[i * dstride + j] = out[i * bw + j];
        }
}

// ---------------------------------------------------------------------------------------------
// distortion: svt_aom_compute_cdef_dist_c / _8bit_c (EbEncCdef.c:129-219), one lane per block
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void cdef_dist_kernel(const T *org, int ost, const T *flt, const SvtGpuCdefList *dl, int n, int bh, int bw,
                                 int luma_ssim, int cs, int ss, unsigned long long *out) {
    const int bi = blockIdx.x * blockDim.x + threadIdx.x;
    if (bi >= n) return;
    const int lbh = bh == 8 ? 3 : 2, lbw = bw == 8 ? 3 : 2;
    const T  *f = flt + (bi << (lbh + lbw));
    const T  *o = org + (dl[bi].by << lbh) * ost + (dl[bi].bx << lbw);
    uint64_t  r = 0;
    if (luma_ssim) {
        uint64_t s1 = 0, d1 = 0, s2 = 0, d2 = 0, sse = 0;
        for (int i = 0; i < 8; i += ss)
            for (int j = 0; j < 8; j++) {
                const uint64_t a = f[8 * i + j], b = o[i * ost + j];
                s1 += a;
                d1 += b;
                s2 += a * a;
                d2 += b * b;
                sse += (a - b) * (a - b);
            }
        r = cdef_luma_dist(s1, d1, s2, d2, sse, cs);
    } else {
        for (int i = 0; i < bh; i += ss)
            for (int j = 0; j < bw; j++) {
                const int e = (int)o[i * ost + j] - (int)f[bw * i + j];
                r += (uint64_t)(e * e);
            }
    }
    atomicAdd(out, (unsigned long long)r);
}

template <typename T>
static uint64_t cdef_dist_host(const T *dst, int32_t dstride, const T *src, const SvtGpuCdefList *dlist, int32_t n,
                               int32_t bsize, int32_t cs, int32_t pli, uint8_t ss) {
    const int bh = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_4X8) ? 8 : 4;
    const int bw = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_8X4) ? 8 : 4;
    const int lbh = bh == 8 ? 3 : 2, lbw = bw == 8 ? 3 : 2;
    if (n <= 0) return 0;
    int maxr = 0, maxc = 0;
    for (int i = 0; i < n; i++) {
        maxr = std::max(maxr, (dlist[i].by + 1) << lbh);
        maxc = std::max(maxc, (dlist[i].bx + 1) << lbw);
    }
    // source region actually read: rows [0, maxr), cols [0, maxc) at stride `dstride`
    std::vector<T> org((size_t)maxr * maxc);
    for (int r = 0; r < maxr; r++) memcpy(&org[(size_t)r * maxc], dst + (long)r * dstride, (size_t)maxc * sizeof(T));
    const size_t fbytes = ((size_t)n << (lbh + lbw)) * sizeof(T);
    const size_t o1 = (org.size() * sizeof(T) + 255) & ~(size_t)255;
    const size_t o2 = o1 + ((fbytes + 255) & ~(size_t)255);
    const size_t o3 = o2 + (((size_t)n * 2 + 255) & ~(size_t)255);
    char        *d  = (char *)g_scratch.get(o3 + 64);
    hipStream_t  st = svtgpu_shim_stream();
    HIP_OR_DIE(hipMemcpyAsync(d, org.data(), org.size() * sizeof(T), hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + o1, src, fbytes, hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + o2, dlist, (size_t)n * 2, hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemsetAsync(d + o3, 0, 8, st));
    const int luma_ssim = bsize == SVTGPU_BLOCK_8X8 && pli == 0;
    hipLaunchKernelGGL(cdef_dist_kernel<T>, dim3((n + 63) / 64), dim3(64), 0, st, (const T *)d, maxc,
                       (const T *)(d + o1), (const SvtGpuCdefList *)(d + o2), n, bh, bw, luma_ssim, cs,
                       ss ? ss : 1, (unsigned long long *)(d + o3));
    HIP_OR_DIE(hipGetLastError());
    uint64_t r = 0;
    HIP_OR_DIE(hipMemcpyAsync(&r, d + o3, 8, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    return r >> (2 * cs);
}

extern "C" uint64_t svtgpu_compute_cdef_dist_16bit(const uint16_t *dst, int32_t dstride, const uint16_t *src,
                                                   const SvtGpuCdefList *dlist, int32_t cdef_count, int32_t bsize,
                                                   int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor) {
    return cdef_dist_host<uint16_t>(dst, dstride, src, dlist, cdef_count, bsize, coeff_shift, pli, subsampling_factor);
}
extern "C" uint64_t svtgpu_compute_cdef_dist_8bit(const uint8_t *dst8, int32_t dstride, const uint8_t *src8,
                                                  const SvtGpuCdefList *dlist, int32_t cdef_count, int32_t bsize,
                                                  int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor) {
    return cdef_dist_host<uint8_t>(dst8, dstride, src8, dlist, cdef_count, bsize, coeff_shift, pli, subsampling_factor);
}

// svt_cdef_filter_block_8xn_16 (AVX2 only in the reference, cdef_block_avx2.c:463-548): rows 0, s, 2s, ... of an
// 8-wide block in steps of two rows (i and i + s per 2s), the same per-sample filter as svt_cdef_filter_block_c
extern "C" void svtgpu_cdef_filter_block_8xn_16(const uint16_t *const in, const int32_t pri_strength,
                                                const int32_t sec_strength, const int32_t dir, int32_t pri_damping,
                                                int32_t sec_damping, const int32_t coeff_shift, uint16_t *const dst,
                                                const int32_t dstride, uint8_t height, uint8_t subsampling_factor) {
    const int ss = subsampling_factor ? subsampling_factor : 1;
    const int bh = (height + 2 * ss - 1) / (2 * ss) * (2 * ss); // the AVX2 loop writes row pairs
    if (bh * 8 > 1024) return;
    const int ws = 8 + 2 * CDEF_BORDER, wh = bh + 2 * CDEF_BORDER;
    std::vector<uint16_t> win((size_t)ws * wh);
    for (int r = 0; r < wh; r++)
        memcpy(&win[(size_t)r * ws], in + (long)(r - CDEF_BORDER) * 144 - CDEF_BORDER, (size_t)ws * 2);
    hipStream_t st   = svtgpu_shim_stream();
    char       *d    = (char *)g_scratch.get(win.size() * 2 + 2 * 1024 + 256);
    uint16_t   *dout = (uint16_t *)(d + ((win.size() * 2 + 15) & ~(size_t)15));
    HIP_OR_DIE(hipMemcpyAsync(d, win.data(), win.size() * 2, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(cdef_filter_block_kernel, dim3(1), dim3(bh * 8), 0, st, (const uint16_t *)d, ws, bh, 8,
                       pri_strength, sec_strength, dir, pri_damping, sec_damping, coeff_shift, ss, dout);
    HIP_OR_DIE(hipGetLastError());
    std::vector<uint16_t> out((size_t)bh * 8);
    HIP_OR_DIE(hipMemcpyAsync(out.data(), dout, out.size() * 2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int i = 0; i < bh; i += ss) memcpy(dst + (long)i * dstride, &out[(size_t)i * 8], 16);
}

// svt_aom_copy_rect8_8bit_to_16bit_c (EbCdef.c:303-311): widen a v x h block of 8-bit samples
__global__ void copy_rect8_kernel(uint16_t *dst, const uint8_t *src, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}
extern "C" void svtgpu_aom_copy_rect8_8bit_to_16bit(uint16_t *dst, int32_t dstride, const uint8_t *src, int32_t sstride,
                                                    int32_t v, int32_t h) {
    if (v <= 0 || h <= 0) return;
    std::vector<uint8_t> hs((size_t)v * h);
    for (int r = 0; r < v; r++) memcpy(&hs[(size_t)r * h], src + (long)r * sstride, (size_t)h);
    hipStream_t st = svtgpu_shim_stream();
    char       *d  = (char *)g_scratch.get(hs.size() * 3 + 64);
    uint16_t   *d16 = (uint16_t *)(d + ((hs.size() + 15) & ~(size_t)15));
    HIP_OR_DIE(hipMemcpyAsync(d, hs.data(), hs.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(copy_rect8_kernel, dim3((unsigned)((hs.size() + 255) / 256)), dim3(256), 0, st, d16,
                       (const uint8_t *)d, (int)hs.size());
    HIP_OR_DIE(hipGetLastError());
    std::vector<uint16_t> out(hs.size());
    HIP_OR_DIE(hipMemcpyAsync(out.data(), d16, out.size() * 2, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int r = 0; r < v; r++) memcpy(dst + (long)r * dstride, &out[(size_t)r * h], (size_t)h * 2);
}

// ---------------------------------------------------------------------------------------------
// svt_search_one_dual_c (EbEncCdef.c:627-695): one lane per (j, k) pair + argmin workgroup
// ---------------------------------------------------------------------------------------------
__global__ void sod_tot_kernel(const uint64_t *mse, int sb, const int32_t *lev, int nb_sel, uint64_t *tot) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x, j = e >> 6, k = e & 63;
    uint64_t  t = 0;
    for (int fb = 0; fb < sb; fb++) {
        const uint64_t *m0 = mse + (size_t)fb * 128, *m1 = m0 + 64;
        uint64_t        best = (uint64_t)1 << 63;
        for (int g = 0; g < nb_sel; g++) {
            const uint64_t c = m0[lev[g]] + m1[lev[16 + g]];
            best = c < best ? c : best;
        }
        const uint64_t c = m0[j] + m1[k];
        t += c < best ? c : best;
    }
    tot[e] = t;
}

__global__ void sod_argmin_kernel(const uint64_t *tot, int start, int end, uint64_t *out) {
    __shared__ uint64_t bv[256];
    __shared__ int32_t  bi[256];
    const int t = threadIdx.x;
    uint64_t  best = (uint64_t)1 << 63;
    int       idx  = 1 << 30;
    for (int u = 0; u < 16; u++) {
        const int e = t * 16 + u, j = e >> 6, k = e & 63;
        if (j >= start && j < end && k >= start && k < end && tot[e] < best) {
            best = tot[e];
            idx  = e;
        }
    }
    bv[t] = best;
    bi[t] = idx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w && (bv[t + w] < bv[t] || (bv[t + w] == bv[t] && bi[t + w] < bi[t]))) {
            bv[t] = bv[t + w];
            bi[t] = bi[t + w];
        }
        __syncthreads();
    }
    if (t == 0) {
        out[0] = bv[0];
        out[1] = bi[0] < (1 << 30) ? (uint64_t)bi[0] : 0;
    }
}

extern "C" uint64_t svtgpu_search_one_dual(int *lev0, int *lev1, int nb_strengths, uint64_t **mse[2], int sb_count,
                                           int start_gi, int end_gi) {
    hipStream_t           st = svtgpu_shim_stream();
    std::vector<uint64_t> h((size_t)std::max(sb_count, 1) * 128);
    for (int fb = 0; fb < sb_count; fb++) {
        memcpy(&h[(size_t)fb * 128], mse[0][fb], 64 * 8);
        memcpy(&h[(size_t)fb * 128 + 64], mse[1][fb], 64 * 8);
    }
    int32_t lev[32] = {0};
    for (int g = 0; g < nb_strengths && g < 16; g++) {
        lev[g]      = lev0[g];
        lev[16 + g] = lev1[g];
    }
    const size_t o1 = h.size() * 8, o2 = o1 + 128, o3 = o2 + 4096 * 8;
    char        *d  = (char *)g_scratch.get(o3 + 16);
    HIP_OR_DIE(hipMemcpyAsync(d, h.data(), h.size() * 8, hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + o1, lev, sizeof lev, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(sod_tot_kernel, dim3(16), dim3(256), 0, st, (const uint64_t *)d, sb_count, (const int32_t *)(d + o1),
                       nb_strengths, (uint64_t *)(d + o2));
    hipLaunchKernelGGL(sod_argmin_kernel, dim3(1), dim3(256), 0, st, (const uint64_t *)(d + o2), start_gi, end_gi,
                       (uint64_t *)(d + o3));
    HIP_OR_DIE(hipGetLastError());
    uint64_t r[2];
    HIP_OR_DIE(hipMemcpyAsync(r, d + o3, 16, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    lev0[nb_strengths] = (int)(r[1] >> 6);
    lev1[nb_strengths] = (int)(r[1] & 63);
    return r[0];
}
