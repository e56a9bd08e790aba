// cdef_apply.hip — apply the picked CDEF strengths to a whole frame (SB64), gfx950.
//
// ≙ svt_av1_cdef_frame (Source/Lib/Encoder/Codec/EbEncCdef.c:284-610).  The reference filters in
// place but reads every neighbour from saved UNFILTERED line/column buffers (:470-547) and 0x7F7F
// outside the frame (:549-568), so the result equals filtering each FB out-of-place from the DLF
// output — which is what this kernel does: one workgroup per 64x64 FB reads its (+-2 px) tile into
// LDS once and writes every output sample of the FB exactly once (filtered, or copied when the FB /
// block / plane is not filtered).  HBM-bound: 1 read + 1 write per sample (+ the 2-px apron).
#include "cdef_common.h"

#define NT 256
#define LT 68
#define CT 36

struct ApplyArgs {
    const void *rec[3];
    void       *out[3];
    int32_t     rstride[3], ostride[3];
    int32_t     width, height, b8_cols, nhfb, cs, fb0, fbw; // filter blocks fb0 + (i / fbw) * nhfb + i % fbw
    int32_t     rect[4];                                    // luma {x0, y0, x1, y1} written (chroma halved)
    const uint8_t *mask;
    const uint8_t *dir;
    const int32_t *var;
    const int8_t  *fb_strength;
    SvtGpuCdefParams prm;
};

template <typename T>
__device__ void stage_tile_a(uint16_t *tile, int ts, int n, const T *plane, int stride, int pw, int ph, int r0, int c0) {
    const int span = n + 2 * CDEF_BORDER;
    for (int i = threadIdx.x; i < span * span; i += NT) {
        const int r = i / span, c = i - r * span;
        const int fr = r0 + r - CDEF_BORDER, fc = c0 + c - CDEF_BORDER;
        uint16_t  v  = CDEF_VERY_LARGE_V;
        if (fr >= 0 && fc >= 0 && fr < ph && fc < pw)
            v = (uint16_t)plane[(long)fr * stride + fc];
        tile[r * ts + c] = v;
    }
}

template <typename T>
__device__ void copy_fb_plane(const T *src, int sst, T *dst, int dst_st, int r0, int c0, int n, const int *lim) {
    for (int i = threadIdx.x; i < n * n; i += NT) {
        const int r = i / n, c = i - r * n;
        if (r0 + r >= lim[1] && r0 + r < lim[3] && c0 + c >= lim[0] && c0 + c < lim[2])
            dst[(long)(r0 + r) * dst_st + c0 + c] = src[(long)(r0 + r) * sst + c0 + c];
    }
}

template <typename T>
__global__ void __launch_bounds__(NT) cdef_apply_kernel(const ApplyArgs A) {
    __shared__ uint16_t ltile[LT * LT];
    __shared__ uint16_t ctile[2][CT * CT];
    __shared__ uint8_t  slisted[64];
    __shared__ int32_t  nlisted;
    const int fi = xcd_swizzle(blockIdx.x, gridDim.x), fb = A.fb0 + (fi / A.fbw) * A.nhfb + fi % A.fbw;
    const int fbr = fb / A.nhfb, fbc = fb - fbr * A.nhfb, tid = threadIdx.x;
    const int cs = A.cs;
    const int si = A.fb_strength[fb];
    int level = A.prm.cdef_y_strength[si] >> 2, sec = A.prm.cdef_y_strength[si] & 3;
    int uvl = A.prm.cdef_uv_strength[si] >> 2, uvs = A.prm.cdef_uv_strength[si] & 3;
    sec += sec == 3; // EbEncCdef.c:390-396
    uvs += uvs == 3;
    if (tid == 0) nlisted = 0;
    __syncthreads();
    if (tid < 64) {
        const int br = 8 * fbr + (tid >> 3), bc = 8 * fbc + (tid & 7);
        const int l = (8 * br < A.height) && (8 * bc < A.width) && (A.mask ? A.mask[br * A.b8_cols + bc] : 1);
        slisted[tid] = (uint8_t)l;
        if (l) atomicAdd(&nlisted, 1);
    }
    __syncthreads();
    const bool fb_on = !(level == 0 && sec == 0 && uvl == 0 && uvs == 0) && nlisted > 0; // :397-402
    const int  pw[3] = {A.width, A.width >> 1, A.width >> 1}, ph[3] = {A.height, A.height >> 1, A.height >> 1};
    for (int pli = 0; pli < 3; pli++) {
        const int n = pli ? 32 : 64, r0 = n * fbr, c0 = n * fbc;
        const T  *src = (const T *)A.rec[pli];
        T        *dst = (T *)A.out[pli];
        const int lv = pli ? uvl : level, sv = pli ? uvs : sec;
        const int sh = pli > 0; // the samples written: the plane clipped to the rect (chroma halved, rounded outward)
        const int lim[4] = {A.rect[0] >> sh, A.rect[1] >> sh, min(pw[pli], (A.rect[2] + sh) >> sh),
                            min(ph[pli], (A.rect[3] + sh) >> sh)};
        if (!fb_on || !(lv || sv)) { // unfiltered plane: pass-through (:404 `level || sec_strength`)
            copy_fb_plane<T>(src, A.rstride[pli], dst, A.ostride[pli], r0, c0, n, lim);
            continue;
        }
        uint16_t *tile = pli ? ctile[pli - 1] : ltile;
        const int ts   = pli ? CT : LT;
        stage_tile_a<T>(tile, ts, n, src, A.rstride[pli], pw[pli], ph[pli], r0, c0);
        __syncthreads();
        const int pri = lv << cs, secs = sv << cs;
        const int damp = A.prm.cdef_damping + cs - (pli != 0);
        const int lb = pli ? 2 : 3;
        for (int i = tid; i < n * n; i += NT) {
            const int r = i / n, c = i - r * n;
            if (r0 + r < lim[1] || r0 + r >= lim[3] || c0 + c < lim[0] || c0 + c >= lim[2]) continue;
            const int b = (r >> lb) * 8 + (c >> lb);
            const uint16_t *p = tile + (r + CDEF_BORDER) * ts + c + CDEF_BORDER;
            int v = p[0];
            if (slisted[b]) {
                const int t = pli ? pri : cdef_adjust_strength(pri, A.var[(size_t)fb * 64 + b]);
                const int d = pri ? A.dir[(size_t)fb * 64 + b] : 0;
                v           = cdef_filter_px(p, ts, t, secs, d, damp, damp, cs);
            }
            dst[(long)(r0 + r) * A.ostride[pli] + c0 + c] = (T)v;
        }
    }
}

int svtgpu_launch_cdef_apply(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, SvtGpuFrame *out,
                             const SvtGpuCdefParams *p, hipStream_t st) {
    ApplyArgs A;
    for (int i = 0; i < 3; i++) {
        A.rec[i]     = recon->plane[i];
        A.out[i]     = out->plane[i];
        A.rstride[i] = recon->stride[i];
        A.ostride[i] = out->stride[i];
    }
    A.width       = recon->width;
    A.height      = recon->height;
    A.b8_cols     = s->geo.b8_cols;
    A.nhfb        = s->geo.nhfb;
    // the filter blocks that hold a sample of the output rect
    const int c0 = s->out_rect[0] / 64, r0 = s->out_rect[1] / 64, c1 = (s->out_rect[2] + 63) / 64,
              r1 = (s->out_rect[3] + 63) / 64;
    A.fb0         = r0 * s->geo.nhfb + c0;
    A.fbw         = c1 - c0;
    for (int i = 0; i < 4; i++) A.rect[i] = s->out_rect[i];
    A.cs          = recon->bit_depth - 8;
    A.mask        = s->mask_all ? nullptr : s->d_mask;
    A.dir         = s->d_dir;
    A.var         = s->d_var;
    A.fb_strength = s->d_fb_strength;
    A.prm         = *p;
    const dim3 grid((r1 - r0) * A.fbw);
    if (recon->bit_depth > 8)
        hipLaunchKernelGGL(cdef_apply_kernel<uint16_t>, grid, dim3(NT), 0, st, A);
    else
        hipLaunchKernelGGL(cdef_apply_kernel<uint8_t>, grid, dim3(NT), 0, st, A);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}
