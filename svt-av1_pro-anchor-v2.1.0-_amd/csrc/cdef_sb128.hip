// cdef_sb128.hip — 128x128 / 128x64 / 64x128 mode-info blocks in the CDEF search tables, gfx950.
//
// With SB128 the reference searches a 128-wide (or tall) block as ONE filter-block area
// (cdef_seg_search, EbCdefProcess.c:188-212): the 64x64 halves at odd FB columns (128x128, 128x64) or odd FB rows
// (128x128, 64x128) are skipped, and the block's list / distortion cover the whole area and land in the entry of
// its top-left 64x64 FB; finish_cdef_search (EbEncCdef.c:805-812) leaves the halves out of the strength pick and
// copies the chosen index into them (:893-909).  The CDEF filter of an 8x8 block reads only its own +-3 samples,
// and the distortion is a sum over listed 8x8 blocks (each scaled by the same subsampling factor), so the area's
// row is the sum of the 64x64 rows our search writes — once the low 2*cs bits each part's shift dropped are added
// back (the reference shifts the area's sum once; the search keeps those bits in d_mse_rem) — except for a chroma
// strength the level does not test, whose entry is the constant default_mse_uv * 64 (EbCdefProcess.c:258-260).
//   fold: per top-left FB of a 128-wide area, sum the rows of its (in-frame) 64x64 parts, skip = AND, and mark the
//         halves skipped so the pick leaves them out;
//   dup:  after the pick, copy the top-left FB's strength index into the halves.
#include "svtgpu_internal.h"

// kind: 0 plain 64x64, 1 128x128, 2 128x64, 3 64x128 (top-left FB of the area), -1 a skipped half
__global__ void __launch_bounds__(64) cdef_sb128_fold_kernel(uint64_t *mse, uint8_t *skip, const uint8_t *rem,
                                                             const int8_t *kind, int nfb, int nhfb, int nvfb,
                                                             unsigned long long uv_on, int cs, int ss, int fb0, int fbw) {
    const int f = fb0 + (blockIdx.x / fbw) * nhfb + blockIdx.x % fbw, k = kind[f], gi = threadIdx.x;
    if (k <= 0) return;
    const int fbr = f / nhfb, fbc = f - fbr * nhfb;
    int       part[4], np = 0;
    part[np++] = f;
    if ((k == 1 || k == 2) && fbc + 1 < nhfb) part[np++] = f + 1;
    if ((k == 1 || k == 3) && fbr + 1 < nvfb) part[np++] = f + nhfb;
    if (k == 1 && fbc + 1 < nhfb && fbr + 1 < nvfb) part[np++] = f + nhfb + 1;
    // the reference shifts the area's summed distortion by 2*cs once (compute_cdef_dist, EbEncCdef.c:129-173);
    // our parts are shifted each: add back what their remainders carry
    uint64_t m0 = 0, m1 = 0;
    uint32_t r0 = 0, r1 = 0, r2 = 0;
    int      all_skip = 1;
    for (int i = 0; i < np; i++) {
        const int p = part[i];
        all_skip &= skip[p] != 0;
        m0 += mse[(size_t)p * 64 + gi];
        m1 += mse[((size_t)nfb + p) * 64 + gi];
        r0 += rem[(size_t)p * 64 + gi];
        r1 += rem[((size_t)nfb + p) * 64 + gi];
        r2 += rem[((size_t)2 * nfb + p) * 64 + gi];
    }
    m0 += (uint64_t)(r0 >> (2 * cs)) * (uint64_t)ss;
    m1 += (uint64_t)(r1 >> (2 * cs)) + (uint64_t)(r2 >> (2 * cs));
    if (!((uv_on >> gi) & 1)) m1 = all_skip ? 0 : 1040400ull * 64; // default_mse_uv * 64
    __syncthreads(); // every lane has read the parts before any is rewritten
    mse[(size_t)f * 64 + gi]           = all_skip ? 0 : m0;
    mse[((size_t)nfb + f) * 64 + gi]   = all_skip ? 0 : m1;
    if (gi == 0) {
        skip[f] = (uint8_t)all_skip;
        for (int i = 1; i < np; i++) skip[part[i]] = 1; // halves: out of the pick (EbEncCdef.c:805-809)
    }
}

__global__ void cdef_sb128_dup_kernel(int8_t *fbs, const int8_t *kind, int nfb, int nhfb, int nvfb) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nfb) return;
    const int k = kind[f];
    if (k <= 0) return;
    const int fbr = f / nhfb, fbc = f - fbr * nhfb, v = fbs[f];
    if ((k == 1 || k == 2) && fbc + 1 < nhfb) fbs[f + 1] = (int8_t)v;
    if ((k == 1 || k == 3) && fbr + 1 < nvfb) fbs[f + nhfb] = (int8_t)v;
    if (k == 1 && fbc + 1 < nhfb && fbr + 1 < nvfb) fbs[f + nhfb + 1] = (int8_t)v;
}

int svtgpu_launch_cdef_sb128_fold(SvtGpuCdefFrameState *s, unsigned long long uv_on, int cs, int ss, hipStream_t st) {
    const int fbw = s->fb_rect[2] - s->fb_rect[0], n = fbw * (s->fb_rect[3] - s->fb_rect[1]);
    if (n > 0)
        hipLaunchKernelGGL(cdef_sb128_fold_kernel, dim3(n), dim3(64), 0, st, s->d_mse, s->d_skip, s->d_mse_rem,
                           s->d_fb_kind, s->nfb, s->geo.nhfb, s->geo.nvfb, uv_on, cs, ss,
                           s->fb_rect[1] * s->geo.nhfb + s->fb_rect[0], fbw);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

int svtgpu_launch_cdef_sb128_dup(SvtGpuCdefFrameState *s, hipStream_t st) {
    hipLaunchKernelGGL(cdef_sb128_dup_kernel, dim3((s->nfb + 255) / 256), dim3(256), 0, st, s->d_fb_strength,
                       s->d_fb_kind, s->nfb, s->geo.nhfb, s->geo.nvfb);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

// host side of the same duplication (the pick's host copy of the per-FB indices)
void svtgpu_cdef_sb128_dup_host(const SvtGpuCdefFrameState *s, int8_t *fbs) {
    const int nhfb = s->geo.nhfb, nvfb = s->geo.nvfb;
    for (int f = 0; f < s->nfb; f++) {
        const int k = s->h_fb_kind[f];
        if (k <= 0) continue;
        const int fbr = f / nhfb, fbc = f - fbr * nhfb;
        if ((k == 1 || k == 2) && fbc + 1 < nhfb) fbs[f + 1] = fbs[f];
        if ((k == 1 || k == 3) && fbr + 1 < nvfb) fbs[f + nhfb] = fbs[f];
        if (k == 1 && fbc + 1 < nhfb && fbr + 1 < nvfb) fbs[f + nhfb + 1] = fbs[f];
    }
}
