// md_dist.hip — mode-decision distortion on gfx950: SAD / SSE / variance for every AV1 block shape.
//
// Reference kernels (Source/Lib/): Encoder/C_DEFAULT/EbComputeSAD_C.c:39-206 (sad, sad_16b_kernel, x4d),
// Encoder/C_DEFAULT/variance.c:256-345 (variance{W}x{H}), Encoder/Codec/EbPsnr.c:146-214
// (highbd_10_variance{W}x{H}), Encoder/Codec/EbEncInterPrediction.c:562-590 (sse / highbd_sse),
// Common/C_DEFAULT/EbPictureOperators_C.c:62 and Common/Codec/EbPictureOperators.c:174 (full distortion).
//
// Batch design (svtgpu_md_dist_batch, round 6): the raw moments of every 4x4 cell -- SAD, signed sum and SSE of the
// differences, additive over cells -- per (SB, reference): one 256-lane workgroup per 64x64 SB, each lane owning one
// 4x4 cell, its 16 source samples in registers across the references (lanes 0-15 of a cell row read 64 consecutive
// samples of a picture row, so each load instruction covers 4 rows x 128 B), one 8-byte store per cell and reference:
// 2 KB per (SB, reference) instead of the 849 x 3 words (10.2 KB) of every shape's values, which wrote more than the
// kernel read (146 MB of outputs against 137 MB of reads per 4K frame, 7 references).  Every shape's SAD, SSE and sum
// are exact sums of its cells' moments, and the reference's variance rounds only the block totals
// (svt_aom_highbd_10_variance*, EbPsnr.c:183-214; variance.c:256-345), so md_expand_kernel derives the [q][849] table of
// an SB range on demand (svtgpu_md_expand / svtgpu_md_read) -- 8 LDS passes, each shape from two halves of a smaller
// one, then the per-bit-depth variance formula.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "svtgpu_internal.h"

namespace {

constexpr int kShapes = SVTGPU_MD_SHAPES;
constexpr int kBlocks = SVTGPU_MD_BLOCKS;
// BlockSize order without the 128 shapes (EbDefinitions.h BlockSize enum); offsets of each shape's blocks
#define MD_W {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 4, 16, 8, 32, 16, 64}
#define MD_H {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 16, 4, 32, 8, 64, 16}
#define MD_OFF {0, 256, 384, 512, 576, 608, 640, 656, 664, 672, 676, 678, 680, 681, 745, 809, 825, 841, 845, 849}
constexpr int    h_w[kShapes] = MD_W, h_h[kShapes] = MD_H, h_off[kShapes + 1] = MD_OFF;
__constant__ int c_w[kShapes] = MD_W, c_h[kShapes] = MD_H, c_off[kShapes + 1] = MD_OFF;

// reduction steps: shape s = two halves of child shape c (horizontally or vertically adjacent);
// steps [c_pass_end[p-1], c_pass_end[p]) depend only on earlier passes
struct Step {
    int s, c, horiz;
};
constexpr int lg2i(int v) { return v <= 1 ? 0 : 1 + lg2i(v / 2); }
// a reduction step with its shifts (every count is a power of two): shape s (output offset off_s) from child shape c
// (offset off_c); blocks of s per SB row 1 << lg_ncol, blocks of s 1 << lg_n, blocks of c per SB row 1 << lg_ccol
struct StepX {
    int16_t off_s, off_c;
    int8_t  lg_ncol, lg_n, lg_ccol, horiz;
};
#define MD_STEP(S, C, HZ)                                                                                          \
    StepX {                                                                                                        \
        (int16_t)h_off[S], (int16_t)h_off[C], (int8_t)lg2i(64 / h_w[S]), (int8_t)lg2i(4096 / (h_w[S] * h_h[S])),     \
            (int8_t)lg2i(64 / h_w[C]), (int8_t)(HZ)                                                                \
    }
__constant__ int  c_pass_end[8] = {2, 5, 7, 10, 12, 15, 17, 18};
__constant__ StepX c_steps[18]  = {
    MD_STEP(2, 0, 1), MD_STEP(1, 0, 0),                    // 8x4, 4x8 from 4x4
    MD_STEP(3, 2, 0), MD_STEP(14, 2, 1), MD_STEP(13, 1, 0), // 8x8, 16x4, 4x16
    MD_STEP(5, 3, 1), MD_STEP(4, 3, 0),                    // 16x8, 8x16
    MD_STEP(6, 5, 0), MD_STEP(16, 5, 1), MD_STEP(15, 4, 0), // 16x16, 32x8, 8x32
    MD_STEP(8, 6, 1), MD_STEP(7, 6, 0),                    // 32x16, 16x32
    MD_STEP(9, 8, 0), MD_STEP(18, 8, 1), MD_STEP(17, 7, 0), // 32x32, 64x16, 16x64
    MD_STEP(11, 9, 1), MD_STEP(10, 9, 0),                  // 64x32, 32x64
    MD_STEP(12, 11, 0),                                    // 64x64
};
#undef MD_STEP

// four samples of a row from x (in the picture, 4 * sizeof(T) bytes): aligned dword loads and a funnel shift (the
// dwords read stay inside [x, x + 3] rounded out to dwords)
template <typename T>
__device__ __forceinline__ void row4(const T *row, int x, int (&v)[4]) {
    const uint32_t *p = (const uint32_t *)((uintptr_t)(row + x) & ~(uintptr_t)3);
    const int       b = (int)((uintptr_t)(row + x) & 3); // byte misalignment
    if constexpr (sizeof(T) == 2) {
        const uint32_t w0 = p[0], w1 = p[1], w2 = p[b ? 2 : 1];
        const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, b * 8), hi = __builtin_amdgcn_alignbit(w2, w1, b * 8);
        v[0] = lo & 0xFFFF, v[1] = lo >> 16, v[2] = hi & 0xFFFF, v[3] = hi >> 16;
    } else {
        const uint32_t w0 = p[0], w1 = p[b ? 1 : 0];
        const uint32_t q = __builtin_amdgcn_alignbyte(w1, w0, b);
        v[0] = q & 0xFF, v[1] = (q >> 8) & 0xFF, v[2] = (q >> 16) & 0xFF, v[3] = q >> 24;
    }
}

struct MdArgs {
    const void    *src;
    int32_t        src_stride;
    const void    *ref[8];
    int32_t        ref_stride[8];
    const int16_t *mv;  // [nsb][nref][2]
    uint2         *mom; // [nsb][nref][256] cell moments
    int32_t        nref, width, height, nsbx, sb_begin, highbd;
};

// cell moments: SAD (<= 16 x 1023, 14 bits) | signed sum (16 bits) << 16, and the SSE (<= 16 x 1023^2 < 2^24)
template <typename T>
__global__ __launch_bounds__(256) void md_dist_kernel(const MdArgs a) {
    const int tid = threadIdx.x;
    const int sb  = a.sb_begin + xcd_swizzle(blockIdx.x, gridDim.x);
    const int ox = (sb % a.nsbx) * 64, oy = (sb / a.nsbx) * 64;
    const int W = a.width, H = a.height;
    const T  *src = (const T *)a.src;
    const bool inside = ox + 64 <= W && oy + 64 <= H;
    const int  cy = tid >> 4, cx = tid & 15;
    int        sv[16]; // the lane's 4x4 source cell, kept for every reference
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int y = oy + cy * 4 + i;
        if (!inside) y = min(y, H - 1);
        const T *row = src + (size_t)y * a.src_stride;
        if (inside) {
            int v[4];
            row4<T>(row, ox + cx * 4, v);
#pragma unroll
            for (int j = 0; j < 4; j++) sv[4 * i + j] = v[j];
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) sv[4 * i + j] = (int)row[min(ox + cx * 4 + j, W - 1)];
        }
    }
    for (int r = 0; r < a.nref; r++) {
        const int mx = a.mv[((size_t)sb * a.nref + r) * 2], my = a.mv[((size_t)sb * a.nref + r) * 2 + 1];
        const T  *ref = (const T *)a.ref[r];
        const int rs  = a.ref_stride[r];
        const int rx = ox + mx, ry = oy + my;
        const bool rin = rx >= 0 && ry >= 0 && rx + 64 <= W && ry + 64 <= H;
        uint32_t   sad = 0, sse = 0;
        int32_t    sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int y = ry + cy * 4 + i;
            if (!rin) y = min(max(y, 0), H - 1);
            const T *row = ref + (size_t)y * rs;
            int      rv[4];
            if (rin) { // the row segment lies inside the picture: aligned dword loads
                row4<T>(row, rx + cx * 4, rv);
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) rv[j] = (int)row[min(max(rx + cx * 4 + j, 0), W - 1)];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = sv[4 * i + j] - rv[j];
                sad += (uint32_t)abs(d);
                sse += (uint32_t)(d * d);
                sum += d;
            }
        }
        a.mom[((size_t)sb * a.nref + r) * 256 + tid] = make_uint2(sad | ((uint32_t)(uint16_t)sum << 16), sse);
    }
}

// every shape's SAD, SSE and variance of (SB, reference) pairs [p0, p0 + grid) from the cell moments
__global__ __launch_bounds__(256) void md_expand_kernel(const uint2 *__restrict__ mom, uint32_t *__restrict__ out,
                                                        size_t p0, int highbd) {
    __shared__ uint32_t s_sad[kBlocks], s_sse[kBlocks];
    __shared__ int32_t  s_sum[kBlocks];
    const int    tid = threadIdx.x;
    const size_t pr  = p0 + blockIdx.x;
    const uint2  m   = mom[pr * 256 + tid];
    s_sad[tid] = m.x & 0xFFFF, s_sse[tid] = m.y, s_sum[tid] = (int32_t)(int16_t)(m.x >> 16);
    // the shape (pixel count) of each output block this lane writes
    constexpr int KO = (kBlocks + 255) / 256;
    int           npx[KO];
#pragma unroll
    for (int j = 0; j < KO; j++) {
        const int k = tid + 256 * j;
        int       sh = 0;
        if (k < kBlocks)
            while (k >= c_off[sh + 1]) sh++;
        npx[j] = c_w[sh] * c_h[sh];
    }
    // hierarchical reduction: 8 passes, each shape from two halves of an already reduced shape
    int st = 0;
    for (int p = 0; p < 8; p++) {
        __syncthreads();
        for (; st < c_pass_end[p]; st++) {
            const StepX q = c_steps[st];
            const int   n = 1 << q.lg_n, mcol = (1 << q.lg_ncol) - 1, ccol = 1 << q.lg_ccol;
            for (int b = tid; b < n; b += 256) {
                const int bi = b >> q.lg_ncol, bj = b & mcol;
                const int c0 = q.horiz ? (bi << q.lg_ccol) + 2 * bj : ((2 * bi) << q.lg_ccol) + bj;
                const int c1 = q.horiz ? c0 + 1 : c0 + ccol;
                const int dst = q.off_s + b, x0 = q.off_c + c0, x1 = q.off_c + c1;
                s_sad[dst] = s_sad[x0] + s_sad[x1];
                s_sse[dst] = s_sse[x0] + s_sse[x1];
                s_sum[dst] = s_sum[x0] + s_sum[x1];
            }
        }
    }
    __syncthreads();
    uint32_t *o = out + pr * 3 * kBlocks;
#pragma unroll
    for (int j = 0; j < KO; j++) {
        const int k = tid + 256 * j;
        if (k >= kBlocks) break;
        const int n = npx[j];
        uint32_t  e, v;
        if (highbd) { // highbd_10_variance: sse rounded >> 4, sum rounded >> 2, clamped at 0
            e                 = (s_sse[k] + 8u) >> 4;
            const int64_t rs2 = ((int64_t)s_sum[k] + 2) >> 2;
            const int64_t var = (int64_t)e - (rs2 * rs2) / n;
            v                 = var >= 0 ? (uint32_t)var : 0u;
        } else {
            e = s_sse[k];
            v = e - (uint32_t)(((int64_t)s_sum[k] * s_sum[k]) / n);
        }
        o[k]               = s_sad[k];
        o[kBlocks + k]     = e;
        o[2 * kBlocks + k] = v;
    }
}

// ---------------------------------------------------------------------------------------------
// per-block shims: Σ|d|, Σd², Σd over nblk compact uint16 blocks (block i of a at a + i*w*h)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void block_stats_kernel(const uint16_t *a, const uint16_t *b, int n,
                                                          unsigned long long *out) {
    __shared__ long long red[3][4];
    const uint16_t *pa = a + (size_t)blockIdx.x * n, *pb = b + (size_t)blockIdx.x * n;
    unsigned long long sad = 0, sse = 0;
    long long          sum = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int d = (int)pa[i] - (int)pb[i];
        sad += (unsigned)abs(d);
        sse += (unsigned long long)((long long)d * d);
        sum += d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        sad += __shfl_down(sad, o, 64);
        sse += __shfl_down(sse, o, 64);
        sum += __shfl_down(sum, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = (long long)sad;
        red[1][threadIdx.x >> 6] = (long long)sse;
        red[2][threadIdx.x >> 6] = sum;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int q = threadIdx.x;
        out[blockIdx.x * 3 + q] = (unsigned long long)(red[q][0] + red[q][1] + red[q][2] + red[q][3]);
    }
}

struct Stats {
    uint64_t sad, sse;
    int64_t  sum;
};

// stage nblk (w x h) blocks (a: 1 block, broadcast; b: nblk blocks) and reduce them on the device
template <typename T>
void block_stats(const T *a, int as, const T *const *b, int bs, int nblk, int w, int h, Stats *out) {
    const int             n = w * h;
    std::vector<uint16_t> ha((size_t)n * nblk), hb((size_t)n * nblk);
    for (int k = 0; k < nblk; k++)
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                ha[(size_t)k * n + y * w + x] = a[(size_t)y * as + x];
                hb[(size_t)k * n + y * w + x] = b[k][(size_t)y * bs + x];
            }
    static thread_local uint16_t *d = nullptr;
    static thread_local size_t    cap = 0;
    static thread_local unsigned long long *dr = nullptr;
    const size_t need = (size_t)2 * n * nblk * sizeof(uint16_t);
    if (need > cap) {
        if (d) (void)hipFree(d);
        HIP_OR_DIE(hipMalloc(&d, need));
        cap = need;
    }
    if (!dr) HIP_OR_DIE(hipMalloc(&dr, sizeof(unsigned long long) * 3 * 4));
    hipStream_t st = svtgpu_shim_stream();
    HIP_OR_DIE(hipMemcpyAsync(d, ha.data(), need / 2, hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + (size_t)n * nblk, hb.data(), need / 2, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(block_stats_kernel, dim3(nblk), dim3(256), 0, st, d, d + (size_t)n * nblk, n, dr);
    HIP_OR_DIE(hipGetLastError());
    unsigned long long r[12];
    HIP_OR_DIE(hipMemcpyAsync(r, dr, sizeof(unsigned long long) * 3 * nblk, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    for (int k = 0; k < nblk; k++) out[k] = {r[3 * k], r[3 * k + 1], (int64_t)r[3 * k + 2]};
}

uint32_t var8(const Stats &s, int n, unsigned int *sse) { // svt_aom_variance{W}x{H}_c
    *sse = (uint32_t)s.sse;
    return *sse - (uint32_t)((s.sum * s.sum) / n);
}
uint32_t var10(const Stats &s, int n, unsigned int *sse) { // svt_aom_highbd_10_variance{W}x{H}_c
    *sse                = (uint32_t)((s.sse + 8) >> 4);
    const int     rsum  = (int)((s.sum + 2) >> 2);
    const int64_t v     = (int64_t)*sse - ((int64_t)rsum * rsum) / n;
    return v >= 0 ? (uint32_t)v : 0u;
}
inline const uint16_t *short_ptr(const uint8_t *p) { return (const uint16_t *)((uintptr_t)p << 1); }

} // namespace

#define MD_SIZE_SHIMS(W, H)                                                                                        \
    extern "C" uint32_t svtgpu_aom_sad##W##x##H(const uint8_t *src, int src_stride, const uint8_t *ref,          \
                                                int ref_stride) {                                                \
        Stats s;                                                                                                 \
        block_stats<uint8_t>(src, src_stride, &ref, ref_stride, 1, W, H, &s);                                     \
        return (uint32_t)s.sad;                                                                                  \
    }                                                                                                            \
    extern "C" void svtgpu_aom_sad##W##x##H##x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[],  \
                                                 int ref_stride, uint32_t *sad_array) {                          \
        Stats s[4];                                                                                              \
        block_stats<uint8_t>(src, src_stride, ref, ref_stride, 4, W, H, s);                                       \
        for (int i = 0; i < 4; i++) sad_array[i] = (uint32_t)s[i].sad;                                           \
    }                                                                                                            \
    extern "C" unsigned int svtgpu_aom_variance##W##x##H(const uint8_t *src, int src_stride, const uint8_t *ref, \
                                                         int ref_stride, unsigned int *sse) {                    \
        Stats s;                                                                                                 \
        block_stats<uint8_t>(src, src_stride, &ref, ref_stride, 1, W, H, &s);                                     \
        return var8(s, W * H, sse);                                                                              \
    }                                                                                                            \
    extern "C" unsigned int svtgpu_aom_highbd_10_variance##W##x##H(const uint8_t *src, int src_stride,           \
                                                                   const uint8_t *ref, int ref_stride,           \
                                                                   unsigned int *sse) {                          \
        Stats           s;                                                                                       \
        const uint16_t *r = short_ptr(ref);                                                                      \
        block_stats<uint16_t>(short_ptr(src), src_stride, &r, ref_stride, 1, W, H, &s);                           \
        return var10(s, W * H, sse);                                                                             \
    }
MD_SIZE_SHIMS(4, 4)
MD_SIZE_SHIMS(4, 8)
MD_SIZE_SHIMS(8, 4)
MD_SIZE_SHIMS(8, 8)
MD_SIZE_SHIMS(8, 16)
MD_SIZE_SHIMS(16, 8)
MD_SIZE_SHIMS(16, 16)
MD_SIZE_SHIMS(16, 32)
MD_SIZE_SHIMS(32, 16)
MD_SIZE_SHIMS(32, 32)
MD_SIZE_SHIMS(32, 64)
MD_SIZE_SHIMS(64, 32)
MD_SIZE_SHIMS(64, 64)
MD_SIZE_SHIMS(64, 128)
MD_SIZE_SHIMS(128, 64)
MD_SIZE_SHIMS(128, 128)
MD_SIZE_SHIMS(4, 16)
MD_SIZE_SHIMS(16, 4)
MD_SIZE_SHIMS(8, 32)
MD_SIZE_SHIMS(32, 8)
MD_SIZE_SHIMS(16, 64)
MD_SIZE_SHIMS(64, 16)

extern "C" uint32_t svtgpu_sad_16b_kernel(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                                          uint32_t height, uint32_t width) {
    Stats           s;
    const uint16_t *r = ref;
    block_stats<uint16_t>(src, (int)src_stride, &r, (int)ref_stride, 1, (int)width, (int)height, &s);
    return (uint32_t)s.sad;
}
extern "C" int64_t svtgpu_aom_sse(const uint8_t *a, int a_stride, const uint8_t *b, int b_stride, int width,
                                  int height) {
    Stats s;
    block_stats<uint8_t>(a, a_stride, &b, b_stride, 1, width, height, &s);
    return (int64_t)s.sse;
}
extern "C" int64_t svtgpu_aom_highbd_sse(const uint8_t *a8, int a_stride, const uint8_t *b8, int b_stride, int width,
                                         int height) {
    Stats           s;
    const uint16_t *b = (const uint16_t *)b8;
    block_stats<uint16_t>((const uint16_t *)a8, a_stride, &b, b_stride, 1, width, height, &s);
    return (int64_t)s.sse;
}
extern "C" uint64_t svtgpu_spatial_full_distortion_kernel(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                                          uint8_t *recon, int32_t recon_offset, uint32_t recon_stride,
                                                          uint32_t area_width, uint32_t area_height) {
    Stats          s;
    const uint8_t *r = recon + recon_offset;
    block_stats<uint8_t>(input + input_offset, (int)input_stride, &r, (int)recon_stride, 1, (int)area_width,
                         (int)area_height, &s);
    return s.sse;
}
extern "C" uint64_t svtgpu_full_distortion_kernel16_bits(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                                         uint8_t *recon, int32_t recon_offset, uint32_t recon_stride,
                                                         uint32_t area_width, uint32_t area_height) {
    Stats           s;
    const uint16_t *r = (const uint16_t *)recon + recon_offset;
    block_stats<uint16_t>((const uint16_t *)input + input_offset, (int)input_stride, &r, (int)recon_stride, 1,
                          (int)area_width, (int)area_height, &s);
    return s.sse;
}

// svt_nxm_sad_kernel / svt_nxm_sad_kernel_sub_sampled (aom_dsp_rtcd.h:853-854): the C versions of both are the
// full N x M SAD (svt_fast_loop_nxm_sad_kernel, EbComputeSAD_C.c:20-37; svt_nxm_sad_kernel_helper_c, :209-212)
extern "C" uint32_t svtgpu_nxm_sad_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                          uint32_t ref_stride, uint32_t height, uint32_t width) {
    Stats s;
    block_stats<uint8_t>(src, (int)src_stride, &ref, (int)ref_stride, 1, (int)width, (int)height, &s);
    return (uint32_t)s.sad;
}
extern "C" uint32_t svtgpu_nxm_sad_kernel_sub_sampled(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                                      uint32_t ref_stride, uint32_t height, uint32_t width) {
    return svtgpu_nxm_sad_kernel(src, src_stride, ref, ref_stride, height, width);
}
// svt_aom_mse16x16_c (EbPsnr.c:76-81): sse - sum^2 / 256, *sse = sse
extern "C" uint32_t svtgpu_aom_mse16x16(const uint8_t *src_ptr, int32_t source_stride, const uint8_t *ref_ptr,
                                        int32_t recon_stride, uint32_t *sse) {
    Stats s;
    block_stats<uint8_t>(src_ptr, source_stride, &ref_ptr, recon_stride, 1, 16, 16, &s);
    return var8(s, 256, sse);
}
// svt_aom_highbd_8_mse16x16_c (variance.c:453-467): *sse = (uint32) sum of squared differences, 16-bit samples
extern "C" void svtgpu_aom_highbd_8_mse16x16(const uint8_t *src_ptr, int32_t source_stride, const uint8_t *ref_ptr,
                                             int32_t recon_stride, uint32_t *sse) {
    Stats           s;
    const uint16_t *r = short_ptr(ref_ptr);
    block_stats<uint16_t>(short_ptr(src_ptr), source_stride, &r, recon_stride, 1, 16, 16, &s);
    *sse = (uint32_t)s.sse;
}
// svt_aom_variance_highbd_c (variance.c:278-296): uint32 sse, int sum, sse - sum^2 / (w*h)
extern "C" uint32_t svtgpu_aom_variance_highbd(const uint16_t *a, int a_stride, const uint16_t *b, int b_stride, int w,
                                               int h, uint32_t *sse) {
    Stats s;
    block_stats<uint16_t>(a, a_stride, &b, b_stride, 1, w, h, &s);
    *sse = (uint32_t)s.sse;
    return (uint32_t)((int64_t)*sse - (s.sum * s.sum) / (w * h));
}

// ---------------------------------------------------------------------------------------------
// svt_aom_sub_pixel_variance{W}x{H}_c (variance.c:308-318): 2-tap bilinear first pass over H+1 rows (u16),
// second pass (u8), then the W x H variance against b.  bilinear_filters_2t[k] = {128 - 16k, 16k}, FILTER_BITS 7.
// One workgroup: the filtered block lives in LDS; the statistics reduce in the workgroup.
// ---------------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void subpel_var_kernel(const uint8_t *a, int as, const uint8_t *b, int w, int h,
                                                         int xoff, int yoff, unsigned long long *out) {
    __shared__ uint16_t f1[129 * 128];
    __shared__ long long red[2][4];
    const int fx0 = 128 - 16 * xoff, fx1 = 16 * xoff, fy0 = 128 - 16 * yoff, fy1 = 16 * yoff;
    for (int i = threadIdx.x; i < (h + 1) * w; i += 256) {
        const int r = i / w, c = i - r * w;
        f1[i] = (uint16_t)(((int)a[r * as + c] * fx0 + (int)a[r * as + c + 1] * fx1 + 64) >> 7);
    }
    __syncthreads();
    unsigned long long sse = 0;
    long long          sum = 0;
    for (int i = threadIdx.x; i < h * w; i += 256) {
        const int v = ((int)f1[i] * fy0 + (int)f1[i + w] * fy1 + 64) >> 7;
        const int d = (int)(uint8_t)v - (int)b[i];
        sse += (unsigned long long)(d * d);
        sum += d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        sse += __shfl_down(sse, o, 64);
        sum += __shfl_down(sum, o, 64);
    }
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = (long long)sse, red[1][threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x < 2) out[threadIdx.x] = (unsigned long long)(red[threadIdx.x][0] + red[threadIdx.x][1] +
                                                                 red[threadIdx.x][2] + red[threadIdx.x][3]);
}

uint32_t subpel_var(const uint8_t *a, int a_stride, int xoff, int yoff, const uint8_t *b, int b_stride, int w, int h,
                    uint32_t *sse) {
    // the first pass reads (h + 1) rows and w + 1 columns of a (the second tap multiplies by 0 at offset 0)
    std::vector<uint8_t> ha((size_t)(h + 1) * (w + 1)), hb((size_t)h * w);
    for (int r = 0; r <= h; r++) memcpy(&ha[(size_t)r * (w + 1)], a + (long)r * a_stride, (size_t)w + 1);
    for (int r = 0; r < h; r++) memcpy(&hb[(size_t)r * w], b + (long)r * b_stride, (size_t)w);
    hipStream_t st = svtgpu_shim_stream();
    static thread_local uint8_t *d = nullptr;
    if (!d) HIP_OR_DIE(hipMalloc(&d, 129 * 129 + 128 * 128 + 64));
    unsigned long long *dr = (unsigned long long *)(d + 129 * 129 + 128 * 128 + 16);
    HIP_OR_DIE(hipMemcpyAsync(d, ha.data(), ha.size(), hipMemcpyHostToDevice, st));
    HIP_OR_DIE(hipMemcpyAsync(d + 129 * 129, hb.data(), hb.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(subpel_var_kernel, dim3(1), dim3(256), 0, st, d, w + 1, d + 129 * 129, w, h, xoff & 7, yoff & 7, dr);
    HIP_OR_DIE(hipGetLastError());
    unsigned long long r[2];
    HIP_OR_DIE(hipMemcpyAsync(r, dr, sizeof r, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    *sse = (uint32_t)r[0];
    return *sse - (uint32_t)(((int64_t)r[1] * (int64_t)r[1]) / (w * h));
}
} // namespace

#define SUBPEL_VAR_SHIM(W, H)                                                                                      \
    extern "C" uint32_t svtgpu_aom_sub_pixel_variance##W##x##H(const uint8_t *src_ptr, int source_stride,          \
                                                               int xoffset, int yoffset, const uint8_t *ref_ptr,   \
                                                               int ref_stride, uint32_t *sse) {                    \
        return subpel_var(src_ptr, source_stride, xoffset, yoffset, ref_ptr, ref_stride, W, H, sse);             \
    }
SUBPEL_VAR_SHIM(4, 4)
SUBPEL_VAR_SHIM(4, 8)
SUBPEL_VAR_SHIM(8, 4)
SUBPEL_VAR_SHIM(8, 8)
SUBPEL_VAR_SHIM(8, 16)
SUBPEL_VAR_SHIM(16, 8)
SUBPEL_VAR_SHIM(16, 16)
SUBPEL_VAR_SHIM(16, 32)
SUBPEL_VAR_SHIM(32, 16)
SUBPEL_VAR_SHIM(32, 32)
SUBPEL_VAR_SHIM(32, 64)
SUBPEL_VAR_SHIM(64, 32)
SUBPEL_VAR_SHIM(64, 64)
SUBPEL_VAR_SHIM(64, 128)
SUBPEL_VAR_SHIM(128, 64)
SUBPEL_VAR_SHIM(128, 128)
SUBPEL_VAR_SHIM(4, 16)
SUBPEL_VAR_SHIM(16, 4)
SUBPEL_VAR_SHIM(8, 32)
SUBPEL_VAR_SHIM(32, 8)
SUBPEL_VAR_SHIM(16, 64)
SUBPEL_VAR_SHIM(64, 16)

// ---------------------------------------------------------------------------------------------
// batch object
// ---------------------------------------------------------------------------------------------
struct SvtGpuMdBatch {
    SvtGpuContext *ctx;
    int32_t        width, height, nref, nsbx, nsby;
    int16_t       *d_mv;
    uint2         *d_mom;  // [nsb][nref][256] cell moments (svtgpu_md_dist_batch)
    uint32_t      *d_out;  // [nsb][nref][3][849] every shape's values (svtgpu_md_expand)
    int32_t        highbd; // the bit depth of the last batch (the expansion's variance formula)
};

extern "C" void svtgpu_md_layout(int32_t *shape_w, int32_t *shape_h, int32_t *shape_offset) {
    for (int s = 0; s < kShapes; s++) {
        if (shape_w) shape_w[s] = h_w[s];
        if (shape_h) shape_h[s] = h_h[s];
        if (shape_offset) shape_offset[s] = h_off[s];
    }
}

extern "C" int svtgpu_md_batch_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t nref,
                                      SvtGpuMdBatch **out) {
    if (!ctx || !out || width <= 0 || height <= 0 || nref < 1 || nref > 8) return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    SvtGpuMdBatch *b = new SvtGpuMdBatch();
    b->ctx           = ctx;
    b->width         = width;
    b->height        = height;
    b->nref          = nref;
    b->nsbx          = (width + 63) / 64;
    b->nsby          = (height + 63) / 64;
    const size_t nsb = (size_t)b->nsbx * b->nsby;
    hipError_t   e   = hipMalloc(&b->d_mv, nsb * nref * 2 * sizeof(int16_t));
    if (e == hipSuccess) e = hipMalloc(&b->d_out, nsb * nref * 3 * kBlocks * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&b->d_mom, nsb * nref * 256 * sizeof(uint2));
    if (e == hipSuccess) e = hipMemset(b->d_mv, 0, nsb * nref * 2 * sizeof(int16_t));
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr); // null-stream memset done before the caller's streams run
    if (e != hipSuccess) {
        svtgpu_md_batch_destroy(b);
        svtgpu_set_last_hip_error(e, "md batch alloc", __FILE__, __LINE__);
        return e == hipErrorOutOfMemory ? SVTGPU_ERR_OOM : SVTGPU_ERR_HIP;
    }
    *out = b;
    return SVTGPU_OK;
}

extern "C" void svtgpu_md_batch_destroy(SvtGpuMdBatch *b) {
    if (!b) return;
    (void)hipFree(b->d_mv);
    (void)hipFree(b->d_out);
    (void)hipFree(b->d_mom);
    delete b;
}

extern "C" int32_t svtgpu_md_batch_nsb(const SvtGpuMdBatch *b) { return b ? b->nsbx * b->nsby : 0; }

extern "C" void *svtgpu_md_out_device_ptr(SvtGpuMdBatch *b) { return b ? b->d_out : nullptr; }

extern "C" int svtgpu_md_set_mvs(SvtGpuMdBatch *b, const int16_t *mv, void *stream) {
    if (!b || !mv) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(b->ctx, stream);
    HIP_TRY(hipMemcpyAsync(b->d_mv, mv, (size_t)b->nsbx * b->nsby * b->nref * 2 * sizeof(int16_t),
                           hipMemcpyHostToDevice, st));
    svtgpu_count_xfer(0, (size_t)b->nsbx * b->nsby * b->nref * 2 * sizeof(int16_t));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

extern "C" int svtgpu_md_dist_batch(SvtGpuMdBatch *b, const SvtGpuFrame *source, const SvtGpuFrame *const *refs,
                                    int32_t sb_begin, int32_t sb_end, void *stream) {
    const int nsb = b ? b->nsbx * b->nsby : 0;
    if (!b || !source || !refs || source->width != b->width || source->height != b->height || sb_begin < 0 ||
        sb_end > nsb || sb_begin > sb_end)
        return SVTGPU_ERR_INVALID_ARG;
    if (source->bit_depth != 8 && source->bit_depth != 10) return SVTGPU_ERR_UNSUPPORTED;
    MdArgs a;
    std::memset(&a, 0, sizeof a);
    a.src        = source->plane[0];
    a.src_stride = source->stride[0];
    for (int r = 0; r < b->nref; r++) {
        const SvtGpuFrame *f = refs[r];
        if (!f || f->width != b->width || f->height != b->height || f->bit_depth != source->bit_depth)
            return SVTGPU_ERR_INVALID_ARG;
        a.ref[r]        = f->plane[0];
        a.ref_stride[r] = f->stride[0];
    }
    a.mv       = b->d_mv;
    a.mom      = b->d_mom;
    a.nref     = b->nref;
    a.width    = b->width;
    a.height   = b->height;
    a.nsbx     = b->nsbx;
    a.sb_begin = sb_begin;
    a.highbd   = source->bit_depth > 8;
    b->highbd  = a.highbd;
    if (sb_end == sb_begin) return SVTGPU_OK;
    hipStream_t st = pick_stream(b->ctx, stream);
    // SVTGPU_MD_LDS=<bytes>: unused dynamic LDS per workgroup, capping how many workgroups share a CU (A/B of the
    // batch's occupancy beside the frames' latency chains)
    static const unsigned lds_pad = [] {
        const char *v = std::getenv("SVTGPU_MD_LDS");
        return v ? (unsigned)std::atoi(v) : 0u;
    }();
    if (a.highbd)
        hipLaunchKernelGGL(md_dist_kernel<uint16_t>, dim3(sb_end - sb_begin), dim3(256), lds_pad, st, a);
    else
        hipLaunchKernelGGL(md_dist_kernel<uint8_t>, dim3(sb_end - sb_begin), dim3(256), lds_pad, st, a);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

extern "C" int svtgpu_md_expand(SvtGpuMdBatch *b, int32_t sb_begin, int32_t sb_end, void *stream) {
    const int nsb = b ? b->nsbx * b->nsby : 0;
    if (!b || sb_begin < 0 || sb_end > nsb || sb_begin > sb_end) return SVTGPU_ERR_INVALID_ARG;
    if (sb_end == sb_begin) return SVTGPU_OK;
    hipLaunchKernelGGL(md_expand_kernel, dim3((sb_end - sb_begin) * b->nref), dim3(256), 0, pick_stream(b->ctx, stream),
                       (const uint2 *)b->d_mom, b->d_out, (size_t)sb_begin * b->nref, (int)b->highbd);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

extern "C" void *svtgpu_md_moments_device_ptr(SvtGpuMdBatch *b) { return b ? (void *)b->d_mom : nullptr; }

extern "C" int svtgpu_md_read(SvtGpuMdBatch *b, uint32_t *out, int32_t sb_begin, int32_t sb_end, void *stream) {
    const int nsb = b ? b->nsbx * b->nsby : 0;
    if (!b || !out || sb_begin < 0 || sb_end > nsb || sb_begin > sb_end) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t  st  = pick_stream(b->ctx, stream);
    if (int rc = svtgpu_md_expand(b, sb_begin, sb_end, st)) return rc; // the rows read, from the moments
    const size_t row = (size_t)b->nref * 3 * kBlocks;
    svtgpu_count_xfer(1, (size_t)(sb_end - sb_begin) * row * sizeof(uint32_t));
    HIP_TRY(hipMemcpyAsync(out, b->d_out + sb_begin * row, (sb_end - sb_begin) * row * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}
