// cdef_apply.hip — apply the picked CDEF strengths to a whole frame (SB64), gfx950.
//
// ≙ svt_av1_cdef_frame (Source/Lib/Encoder/Codec/EbEncCdef.c:284-610).  The reference filters in
// place but reads every neighbour from saved UNFILTERED line/column buffers (:470-547) and 0x7F7F
// outside the frame (:549-568), so the result equals filtering each FB out-of-place from the DLF
// output — which is what this kernel does: one workgroup per 64x64 FB reads its (+-2 px) tile into
// LDS once and writes every output sample of the FB exactly once (filtered, or copied when the FB /
// block / plane is not filtered).  1 read + 1 write per sample (+ the 2-px apron); ~130 integer ops per filtered
// sample, done two samples per lane on packed int16.
#include <cstring>

#include "cdef_common.h"

#define NT 256
// LDS tiles: the FB's n x n samples at column TC0 of each row (16-B aligned rows, so the interior is written with one
// 16-B store per 8 samples), the +-2 px apron around them
#define TC0 8
#define LT 80 // luma row stride (samples): TC0 + 64 + 2, rounded up to 8
#define CT 48 // chroma
#define LR 68 // luma rows: 64 + 2 * 2
#define CR 36

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
    const SvtGpuCdefParams *dprm; // the asynchronous pick's parameters in device memory (read instead of prm), or null
    unsigned long long *wgclk; // diagnostics (svtgpu_internal.h wgclk_mark) or null
};

// 8 samples of a row from (fr, fc) as 16-bit values, 0x7F7F (CDEF_VERY_LARGE_V) outside the plane: one 16-B (8-B)
// load; the rows are padded to 256 B, so a segment that starts inside the plane reads only its own row
template <typename T>
__device__ __forceinline__ uint4 load_seg8(const T *plane, int stride, int pw, int ph, int fr, int fc) {
    uint4 w = {0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu, 0x7F7F7F7Fu};
    if (fr < 0 || fr >= ph || fc >= pw) return w;
    const T *src = plane + (long)fr * stride + fc;
    if constexpr (sizeof(T) == 2) {
        w = *(const uint4 *)src;
    } else {
        const uint2 b = *(const uint2 *)src;
        w.x = (b.x & 0xFF) | ((b.x & 0xFF00) << 8), w.y = ((b.x >> 16) & 0xFF) | ((b.x >> 8) & 0xFF0000);
        w.z = (b.y & 0xFF) | ((b.y & 0xFF00) << 8), w.w = ((b.y >> 16) & 0xFF) | ((b.y >> 8) & 0xFF0000);
    }
    if (fc + 8 > pw) { // the plane's last segment of a row (chroma widths of 4 mod 8)
        uint32_t *q = &w.x;
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (fc + j >= pw) q[j >> 1] = (j & 1) ? (q[j >> 1] & 0xFFFFu) | 0x7F7F0000u : (q[j >> 1] & 0xFFFF0000u) | 0x7F7Fu;
    }
    return w;
}

// Stage the n x n FB at (r0, c0) with its 2-px apron: every interior 8-sample row segment one vector load and one
// 16-B LDS store (all of a lane's loads issued before the first store), the apron columns one sample each
template <typename T, int N>
__device__ __forceinline__ void stage_tile_v(uint16_t *tile, const T *plane, int stride, int pw, int ph, int r0, int c0) {
    constexpr int TS = N == 64 ? LT : CT, ROWS = N + 4, SEGS = N / 8, NI = ROWS * SEGS, IT = (NI + NT - 1) / NT;
    uint4 v[IT];
#pragma unroll
    for (int u = 0; u < IT; u++) {
        const int i = threadIdx.x + u * NT, r = i / SEGS, sg = i % SEGS;
        if (i < NI) v[u] = load_seg8<T>(plane, stride, pw, ph, r0 + r - CDEF_BORDER, c0 + 8 * sg);
    }
    constexpr int NB = ROWS * 4, IB = (NB + NT - 1) / NT; // apron: 2 columns each side per row
    uint16_t      b[IB];
    int           bo[IB];
#pragma unroll
    for (int u = 0; u < IB; u++) {
        const int i = threadIdx.x + u * NT, r = i >> 2, k = i & 3, dc = k < 2 ? k - 2 : N + k - 2;
        const int fr = r0 + r - CDEF_BORDER, fc = c0 + dc;
        b[u]  = CDEF_VERY_LARGE_V;
        bo[u] = r * TS + TC0 + dc;
        if (i < NB && fr >= 0 && fr < ph && fc >= 0 && fc < pw) b[u] = (uint16_t)plane[(long)fr * stride + fc];
    }
#pragma unroll
    for (int u = 0; u < IT; u++) {
        const int i = threadIdx.x + u * NT, r = i / SEGS, sg = i % SEGS;
        if (i < NI) *(uint4 *)(tile + r * TS + TC0 + 8 * sg) = v[u];
    }
#pragma unroll
    for (int u = 0; u < IB; u++)
        if (threadIdx.x + u * NT < NB) tile[bo[u]] = b[u];
}

// Two horizontally adjacent output samples (the pair at p, p + 1 of a tile; one block) of svt_cdef_filter_block_c
// (EbCdef.c:253-300) on packed int16 lanes: the primary taps (offsets op_k, +-) with threshold `pthr` (strength-
// adjusted, shift psh) and weights pw0 / pw1 ({4, 2} or {3, 3}), the secondary taps (o0_k, o1_k, +-) with sthr /
// ssh and weights {2, 1}, then the clamp to the taps' range.  `ofs` holds the block's tap offsets (int16 halves:
// k = 0 low, k = 1 high) for op, o0, o1.  constrain(d, thr, damping) = sign(d) * min(|d|, m) with
// m = max(0, thr - (|d| >> shift)) >= 0 is the clamp of d to [-m, m].  EDGE: taps outside the frame (0x7F7F, bit 14
// set; samples stay below 2^12) are left out of the maximum -- not needed for an FB whose apron is inside the
// frame.  The int16 sums wrap exactly as the reference's int16_t sum.
// The pair of samples at 16-bit index a of an LDS tile from two aligned dwords (one ds_read2_b32) and a funnel
// shift: a dword read at an odd sample index is a misaligned LDS access, which the LDS serves far below its rate.
__device__ __forceinline__ s16x2 lds_pair(const uint16_t *tile, int a) {
    const uint32_t *w = (const uint32_t *)tile + (a >> 1);
    return __builtin_bit_cast(s16x2, __builtin_amdgcn_alignbit(w[1], w[0], (a & 1) * 16));
}

template <bool EDGE>
__device__ __forceinline__ s16x2 cdef_filter_pair(const uint16_t *tile, int a0, uint4 ofs, s16x2 pthr, u16x2 psh,
                                                  s16x2 pw0, s16x2 pw1, s16x2 sthr, u16x2 ssh) {
    const s16x2 x  = __builtin_bit_cast(s16x2, *(const uint32_t *)(tile + a0)); // a0 is even
    s16x2       lo = x, hi = x, sum = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int op = (int)(int16_t)(k ? ofs.x >> 16 : ofs.x), o0 = (int)(int16_t)(k ? ofs.y >> 16 : ofs.y),
                  o1 = (int)(int16_t)(k ? ofs.z >> 16 : ofs.z);
        const int o[6] = {op, -op, o0, -o0, o1, -o1};
        s16x2     ps = {0, 0}, ss = {0, 0};
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const s16x2 v  = lds_pair(tile, a0 + o[t]);
            const s16x2 d  = v - x;
            const s16x2 ad = __builtin_elementwise_max(d, (s16x2){0, 0} - d);
            lo = __builtin_elementwise_min(lo, v);
            if (EDGE) {
                const s16x2 out = (s16x2)((u16x2)v >> (u16x2){14, 14});
                hi = __builtin_elementwise_max(hi, v & (out - (s16x2){1, 1}));
            } else {
                hi = __builtin_elementwise_max(hi, v);
            }
            const s16x2 m = __builtin_elementwise_max((t < 2 ? pthr : sthr) - (s16x2)((u16x2)ad >> (t < 2 ? psh : ssh)),
                                                      (s16x2){0, 0});
            const s16x2 c = __builtin_elementwise_max(__builtin_elementwise_min(d, m), (s16x2){0, 0} - m);
            if (t < 2) ps = ps + c;
            else ss = ss + c;
        }
        sum = sum + ps * (k ? pw1 : pw0) + ss * (k ? (s16x2){1, 1} : (s16x2){2, 2});
    }
    const s16x2 rnd = (sum + (s16x2){8, 8} + (sum >> (s16x2){15, 15})) >> (s16x2){4, 4};
    return __builtin_elementwise_max(__builtin_elementwise_min(x + rnd, hi), lo);
}

// the tap offsets of direction `dir` in a tile of row stride ts, packed as cdef_filter_pair reads them
__device__ __forceinline__ uint4 cdef_tap_offsets(int dir, int ts) {
    const int ds0 = (dir + 2) & 7, ds1 = (dir + 6) & 7;
    uint32_t  w[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int o[3] = {cdef_dir_dy(dir, k) * ts + cdef_dir_dx(dir, k), cdef_dir_dy(ds0, k) * ts + cdef_dir_dx(ds0, k),
                          cdef_dir_dy(ds1, k) * ts + cdef_dir_dx(ds1, k)};
#pragma unroll
        for (int q = 0; q < 3; q++) w[q] |= (uint32_t)(uint16_t)o[q] << (16 * k);
    }
    return (uint4){w[0], w[1], w[2], 0u};
}

// One workgroup per FB: the filtered planes' tiles staged together (one barrier), then every lane writes 8-sample
// row segments (luma 512, chroma 2 x 128 per FB) as four packed pairs with one vector store each segment.
template <typename T>
__global__ void __launch_bounds__(NT) cdef_apply_kernel(const ApplyArgs A) {
    __shared__ __attribute__((aligned(16))) uint16_t ltile[LR * LT];
    __shared__ __attribute__((aligned(16))) uint16_t ctile[2][CR * CT];
    __shared__ uint8_t  slisted[64];
    __shared__ uint32_t sadj[64];    // luma: the block's variance-adjusted primary strength | its shift << 16
    __shared__ uint4    sofs[2][64]; // the block's tap offsets in the luma / chroma tile
    __shared__ int32_t  nlisted;
    wgclk_mark(A.wgclk, 0);
    const int fi = xcd_swizzle(blockIdx.x, gridDim.x), fb = A.fb0 + (fi / A.fbw) * A.nhfb + fi % A.fbw;
    const int fbr = fb / A.nhfb, fbc = fb - fbr * A.nhfb, tid = threadIdx.x;
    const int cs = A.cs;
    const int si = A.fb_strength[fb];
    const int ycode = A.dprm ? A.dprm->cdef_y_strength[si] : A.prm.cdef_y_strength[si];
    const int uvcode = A.dprm ? A.dprm->cdef_uv_strength[si] : A.prm.cdef_uv_strength[si];
    const int damping = A.dprm ? A.dprm->cdef_damping : A.prm.cdef_damping;
    int level = ycode >> 2, sec = ycode & 3;
    int uvl = uvcode >> 2, uvs = uvcode & 3;
    sec += sec == 3; // EbEncCdef.c:390-396
    uvs += uvs == 3;
    if (tid == 0) nlisted = 0;
    __syncthreads();
    if (tid < 64) {
        const int br = 8 * fbr + (tid >> 3), bc = 8 * fbc + (tid & 7);
        const int l = (8 * br < A.height) && (8 * bc < A.width) && (A.mask ? A.mask[br * A.b8_cols + bc] : 1);
        slisted[tid]  = (uint8_t)l;
        const int dir = l ? A.dir[(size_t)fb * 64 + tid] : 0; // pri_strength ? dir : 0 (EbCdef.c:404)
        const int t   = l ? cdef_adjust_strength(level << cs, A.var[(size_t)fb * 64 + tid]) : 0;
        sadj[tid]     = (uint32_t)t | ((uint32_t)max(0, damping + cs - msb32_dev((uint32_t)t)) << 16);
        sofs[0][tid]  = cdef_tap_offsets(level ? dir : 0, LT);
        sofs[1][tid]  = cdef_tap_offsets(uvl ? dir : 0, CT);
        if (l) atomicAdd(&nlisted, 1);
    }
    __syncthreads();
    wgclk_mark(A.wgclk, 1);
    const bool fb_on = !(level == 0 && sec == 0 && uvl == 0 && uvs == 0) && nlisted > 0; // :397-402
    const int  pw[3] = {A.width, A.width >> 1, A.width >> 1}, ph[3] = {A.height, A.height >> 1, A.height >> 1};
    bool       on[3];
#pragma unroll
    for (int pli = 0; pli < 3; pli++) { // filtered planes: stage their tiles (:404 `level || sec_strength`)
        on[pli] = fb_on && (pli ? (uvl || uvs) : (level || sec));
        if (!on[pli]) continue;
        if (pli == 0)
            stage_tile_v<T, 64>(ltile, (const T *)A.rec[0], A.rstride[0], pw[0], ph[0], 64 * fbr, 64 * fbc);
        else
            stage_tile_v<T, 32>(ctile[pli - 1], (const T *)A.rec[pli], A.rstride[pli], pw[pli], ph[pli], 32 * fbr,
                                32 * fbc);
    }
    __syncthreads();
    wgclk_mark(A.wgclk, 2);
    // planes not filtered: 8-sample row segments copied with one vector load / store each
    for (int sgi = tid; sgi < 512 + 2 * 128; sgi += NT) {
        const int pli = sgi < 512 ? 0 : 1 + ((sgi - 512) >> 7), loc = pli ? (sgi - 512) & 127 : sgi;
        if (on[pli]) continue;
        const int n = pli ? 32 : 64, spr = n >> 3, r = loc / spr, c0 = 8 * (loc - r * spr);
        const int sh = pli > 0;
        const int lim[4] = {A.rect[0] >> sh, A.rect[1] >> sh, min(pw[pli], (A.rect[2] + sh) >> sh),
                            min(ph[pli], (A.rect[3] + sh) >> sh)};
        const int y = n * fbr + r, x0 = n * fbc + c0;
        if (y < lim[1] || y >= lim[3] || x0 + 8 <= lim[0] || x0 >= lim[2]) continue;
        const T *src = (const T *)A.rec[pli] + (long)y * A.rstride[pli] + x0;
        T       *dst = (T *)A.out[pli] + (long)y * A.ostride[pli] + x0;
        if (x0 >= lim[0] && x0 + 8 <= lim[2]) { // whole segment inside (lim[2] <= pw)
            if constexpr (sizeof(T) == 2)
                *(uint4 *)dst = *(const uint4 *)src;
            else
                *(uint2 *)dst = *(const uint2 *)src;
        } else {
            for (int j = 0; j < 8; j++)
                if (x0 + j >= lim[0] && x0 + j < lim[2]) dst[j] = src[j];
        }
    }
    wgclk_mark(A.wgclk, 3);
    // filtered planes: one horizontal pair of samples per lane, consecutive lanes along a row -- a wave's LDS reads
    // of one tap cover 32 consecutive words per tile row (2 lanes per bank, the b32 minimum), and its stores are
    // whole rows (luma 2048 pairs, chroma 2 x 512).  An FB whose 2-px apron lies inside the frame has no 0x7F7F taps.
    const bool interior = fbr > 0 && fbc > 0 && 64 * fbr + 68 <= A.height && 64 * fbc + 68 <= A.width; // chroma: +34
#pragma unroll
    for (int pli = 0; pli < 3; pli++) {
        if (!on[pli]) continue;
        const int n = pli ? 32 : 64, lp = pli ? 4 : 5, lb = pli ? 2 : 3, ts = pli ? CT : LT, sh = pli > 0;
        const int xlo = A.rect[0] >> sh, ylo = A.rect[1] >> sh, xhi = min(pw[pli], (A.rect[2] + sh) >> sh),
                  yhi = min(ph[pli], (A.rect[3] + sh) >> sh);
        const uint16_t *tile = pli ? ctile[pli - 1] : ltile;
        // plane-uniform strengths: the chroma primary (no variance adjustment, EbCdef.c:401) and the secondary
        const int   damp = damping + cs - (pli != 0);
        const int   cpri = uvl << cs, secs = (pli ? uvs : sec) << cs, podd_c = (cpri >> cs) & 1;
        const s16x2 sthr = {(short)secs, (short)secs};
        const unsigned short ss = (unsigned short)max(0, damp - msb32_dev((uint32_t)secs)),
                             cs_sh = (unsigned short)max(0, damp - msb32_dev((uint32_t)cpri));
        const u16x2 ssh = {ss, ss};
        T *out = (T *)A.out[pli];
        for (int j = tid; j < (n * n) >> 1; j += NT) {
            // luma: a half-wave is one tile row (32 pairs); chroma: a half-wave holds two rows of 16 pairs, taken two
            // apart (r, r + 2: 48 dwords, disjoint banks; adjacent rows, 24 dwords apart, shared 8 banks pairwise)
            const int r = pli ? ((j >> 6) << 2) | (((j >> 4) & 1) << 1) | ((j >> 5) & 1) : j >> lp;
            const int c = 2 * (j & ((1 << lp) - 1));
            const int y = n * fbr + r, x = n * fbc + c;
            if (y < ylo || y >= yhi || x < xlo || x >= xhi) continue; // x bounds are even: a pair is in or out whole
            const int       b = (r >> lb) * 8 + (c >> lb);
            const int       a0 = (r + CDEF_BORDER) * ts + c + TC0; // even: ts, c and TC0 are
            s16x2           v  = __builtin_bit_cast(s16x2, *(const uint32_t *)(tile + a0));
            if (slisted[b]) {
                int t = cpri, psh = cs_sh, podd = podd_c;
                if (!pli) {
                    const uint32_t a = sadj[b];
                    t = (int)(a & 0xFFFF), psh = (int)(a >> 16), podd = (t >> cs) & 1;
                }
                const s16x2 pthr = {(short)t, (short)t};
                const u16x2 pshv = {(unsigned short)psh, (unsigned short)psh};
                const s16x2 pw0 = podd ? (s16x2){3, 3} : (s16x2){4, 4}, pw1 = podd ? (s16x2){3, 3} : (s16x2){2, 2};
                const uint4 ofs = sofs[pli != 0][b];
                v = interior ? cdef_filter_pair<false>(tile, a0, ofs, pthr, pshv, pw0, pw1, sthr, ssh)
                             : cdef_filter_pair<true>(tile, a0, ofs, pthr, pshv, pw0, pw1, sthr, ssh);
            }
            T *dst = out + (long)y * A.ostride[pli] + x;
            if constexpr (sizeof(T) == 2)
                *(uint32_t *)dst = (uint32_t)(uint16_t)v.x | ((uint32_t)(uint16_t)v.y << 16);
            else
                *(uint16_t *)dst = (uint16_t)((uint8_t)v.x | ((uint8_t)v.y << 8));
        }
    }
    if (A.wgclk) {
        __syncthreads();
        wgclk_mark(A.wgclk, 5);
    }
}

__global__ void cdef_set_params_kernel(SvtGpuCdefParams *d, const SvtGpuCdefParams p) {
    if (threadIdx.x == 0) *d = p;
}
int svtgpu_launch_cdef_set_params(SvtGpuCdefFrameState *s, const SvtGpuCdefParams *p, hipStream_t st) {
    hipLaunchKernelGGL(cdef_set_params_kernel, dim3(1), dim3(64), 0, st, (SvtGpuCdefParams *)((uint8_t *)s->d_apick + 16), *p);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
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
    if (p) A.prm = *p;
    else std::memset(&A.prm, 0, sizeof A.prm);
    A.dprm        = p ? nullptr : (const SvtGpuCdefParams *)((const uint8_t *)s->d_apick + 16);
    const dim3 grid((r1 - r0) * A.fbw);
    A.wgclk = svtgpu_wgclk_begin((int)grid.x);
    if (recon->bit_depth > 8)
        hipLaunchKernelGGL(cdef_apply_kernel<uint16_t>, grid, dim3(NT), 0, st, A);
    else
        hipLaunchKernelGGL(cdef_apply_kernel<uint8_t>, grid, dim3(NT), 0, st, A);
    HIP_TRY(hipGetLastError());
    svtgpu_wgclk_end("cdef_apply", (int)grid.x, st);
    return SVTGPU_OK;
}
