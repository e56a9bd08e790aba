// me_sad.hip — open-loop motion-estimation SAD kernels on gfx950.
//
// Reference: Source/Lib/Encoder/Codec/EbMotionEstimation.c — the full-pel search of one 64x64 block
// (open_loop_me_fullpel_search_sblock, :782-818) over svt_ext_all_sad_calculation_8x8_16x16 (:336-368) +
// svt_ext_eight_sad_calculation_32x32_64x64 (:370-428) for every 8 horizontal positions and the single-point
// svt_ext_sad_calculation_8x8_16x16 (:99-170) + svt_ext_sad_calculation_32x32_64x64 (:172-210) for the rest of a row;
// svt_sad_loop_kernel_c (Source/Lib/Encoder/C_DEFAULT/EbComputeSAD_C.c:58-99).
//
// Frame level (svtgpu_me_search): one workgroup per (64x64 block, reference).  Lane L of each wave owns the 8x8 block
// of Z-order index L (the reference's 8x8 / 16x16 numbering: 16x16 q = L >> 2 in Z-order, 8x8 sub = L & 3 raster
// inside it), its source rows live in registers; the wave's four 16x16 / 32x32 / 64x64 sums are lane-group
// reductions (4, 16, 64 lanes).  The reference window of a band of 32 search rows is staged in LDS; wave w takes the
// search rows y = w (mod 4), each lane walks x in groups of 4 positions: per block row it reads 3 dwords of the window
// and forms the 4 unaligned 8-byte rows with v_alignbyte, so one v_sad_u8 pair per row per position.  Per lane the best
// (SAD, scan index) of each of its four block levels is kept with the reference's strict "<" in scan order (y, then
// x), and the four waves' results are merged lexicographically -- the first minimum of the reference's scan.
// Samples outside the reference frame read the nearest edge sample: the encoder's reference pictures are padded by
// edge replication (svt_aom_generate_padding, EbMcp.c:95-150), so any search inside the padding reads the same values.
#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "svtgpu_internal.h"

namespace {

constexpr uint32_t kMaxSad   = 128 * 128 * 255; // MAX_SAD_VALUE (EbMotionEstimation.h:94): the initial best
constexpr int      kBand     = 32;              // search rows per staged reference window
constexpr int      kMaxSaw   = 192;             // widest search area per launch (window row 64 + 191 + slack)
constexpr int      kWinCols  = 64 + kMaxSaw + 8;
constexpr int      kWinRows  = 64 + kBand - 1;
constexpr int      kOut      = 85; // 64 8x8 + 16 16x16 + 4 32x32 + 1 64x64

struct MeArgs {
    const uint8_t *src;
    int32_t        src_stride, width, height, nsbx, nref, sb_begin;
    const uint8_t *ref[8];
    int32_t        ref_stride[8];
    const int16_t *origin; // [nsb][nref][2] search-area origin (x, y) relative to the block
    int32_t        saw, sah, sub;
    uint32_t      *best_sad, *best_mv; // [nsb][nref][85]
};

__device__ inline uint32_t sad4(uint32_t a, uint32_t b, uint32_t acc) { return __builtin_amdgcn_sad_u8(a, b, acc); }
__device__ inline uint32_t align4(uint32_t hi, uint32_t lo, int s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

// (x, y) of the 8x8 block of Z-order index L inside the 64x64 block
__device__ inline void z8(int L, int &bx, int &by) {
    const int q = L >> 2, k = q >> 2, s = L & 3;
    bx = 32 * (k & 1) + 16 * (q & 1) + 8 * (s & 1);
    by = 32 * (k >> 1) + 16 * ((q >> 1) & 1) + 8 * (s >> 1);
}

// sum over aligned groups of `width` lanes of a value already equal within groups of `from` lanes
__device__ inline uint32_t lane_sum(uint32_t v, int from, int width) {
    for (int o = from; o < width; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

struct Best {
    uint32_t sad, idx;
    __device__ void take(uint32_t s, uint32_t i) { // strict "<": the earlier scan position keeps a tie
        if (s < sad) sad = s, idx = i;
    }
    __device__ void merge(uint32_t s, uint32_t i) { // lexicographic (SAD, scan index) minimum
        if (s < sad || (s == sad && i < idx)) sad = s, idx = i;
    }
};

__global__ __launch_bounds__(256) void me_search_kernel(const MeArgs A) {
    __shared__ __align__(16) uint8_t win[kWinRows * kWinCols];
    __shared__ uint32_t             wb[4][4][64][2]; // per wave, level, lane: (sad, idx)
    const int task = A.sb_begin * A.nref + blockIdx.x, sb = task / A.nref, r = task % A.nref;
    const int sx0 = 64 * (sb % A.nsbx), sy0 = 64 * (sb / A.nsbx);
    const int ox = A.origin[2 * task], oy = A.origin[2 * task + 1];
    const int L = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint8_t *ref = A.ref[r];
    const int      rs  = A.ref_stride[r];
    int bx, by;
    z8(L, bx, by);
    // this lane's 8x8 source block (rows 0, 2, 4, 6 only when sub-sampled), edge-clamped
    uint32_t s0[8], s1[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int y = min(sy0 + by + k, A.height - 1);
        uint32_t  v[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int x = min(sx0 + bx + c, A.width - 1);
            v[c >> 2] |= (uint32_t)A.src[(size_t)y * A.src_stride + x] << (8 * (c & 3));
        }
        s0[k] = v[0], s1[k] = v[1];
    }
    Best b[4];
#pragma unroll
    for (int l = 0; l < 4; l++) b[l].sad = 0xFFFFFFFFu, b[l].idx = 0xFFFFFFFFu;
    const int wcols = 64 + A.saw - 1, wpad = (wcols + 3 + 3) & ~3; // + the 3 bytes the last group over-reads
    for (int y0 = 0; y0 < A.sah; y0 += kBand) {
        const int rows = min(kBand, A.sah - y0) + 63;
        __syncthreads(); // the previous band's window is no longer read
        for (int i = threadIdx.x; i < rows * (wpad >> 2); i += 256) {
            const int rr = i / (wpad >> 2), cq = i - rr * (wpad >> 2);
            const int y  = min(max(sy0 + oy + y0 + rr, 0), A.height - 1);
            uint32_t  v  = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int x = min(max(sx0 + ox + 4 * cq + c, 0), A.width - 1);
                v |= (uint32_t)ref[(size_t)y * rs + x] << (8 * c);
            }
            *(uint32_t *)(win + rr * kWinCols + 4 * cq) = v;
        }
        __syncthreads();
        for (int yy = w; yy < min(kBand, A.sah - y0); yy += 4) {
            for (int x0 = 0; x0 < A.saw; x0 += 4) {
                uint32_t sad[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    if (A.sub && (k & 1)) continue;
                    const uint32_t *row = (const uint32_t *)(win + (yy + by + k) * kWinCols + x0 + bx);
                    const uint32_t  d0 = row[0], d1 = row[1], d2 = row[2];
#pragma unroll
                    for (int s = 0; s < 4; s++)
                        sad[s] = sad4(s1[k], align4(d2, d1, s), sad4(s0[k], align4(d1, d0, s), sad[s]));
                }
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const uint32_t v8 = A.sub ? sad[s] << 1 : sad[s];
                    const uint32_t v16 = lane_sum(v8, 1, 4), v32 = lane_sum(v16, 4, 16), v64 = lane_sum(v32, 16, 64);
                    if (x0 + s < A.saw) {
                        const uint32_t idx = (uint32_t)(y0 + yy) * (uint32_t)A.saw + (uint32_t)(x0 + s);
                        b[0].take(v8, idx), b[1].take(v16, idx), b[2].take(v32, idx), b[3].take(v64, idx);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int l = 0; l < 4; l++) wb[w][l][L][0] = b[l].sad, wb[w][l][L][1] = b[l].idx;
    __syncthreads();
    if (w) return;
#pragma unroll
    for (int l = 0; l < 4; l++)
        for (int ww = 1; ww < 4; ww++) b[l].merge(wb[ww][l][L][0], wb[ww][l][L][1]);
    // outputs: 8x8 [64], 16x16 [16], 32x32 [4], 64x64 [1]; MAX_SAD_VALUE / mv 0 stay when nothing is below them
    uint32_t *os = A.best_sad + (size_t)task * kOut, *om = A.best_mv + (size_t)task * kOut;
    auto put = [&](int o, const Best &v) {
        const bool hit = v.sad < kMaxSad;
        const int  x = hit ? (int)(v.idx % (uint32_t)A.saw) : 0, y = hit ? (int)(v.idx / (uint32_t)A.saw) : 0;
        os[o] = hit ? v.sad : kMaxSad;
        om[o] = hit ? ((uint32_t)(uint16_t)(oy + y) << 16) | (uint32_t)(uint16_t)(ox + x) : 0u;
    };
    put(L, b[0]);
    if ((L & 3) == 0) put(64 + (L >> 2), b[1]);
    if ((L & 15) == 0) put(80 + (L >> 4), b[2]);
    if (L == 0) put(84, b[3]);
}

// ---- per-call RTCD kernels (one small launch each) ----
__device__ inline uint32_t sad8x8(const uint8_t *s, int ss, const uint8_t *r, int rs, bool sub) {
    uint32_t a = 0;
    for (int y = 0; y < 8; y += sub ? 2 : 1)
        for (int x = 0; x < 8; x++) a += (uint32_t)abs((int)s[y * ss + x] - (int)r[y * rs + x]);
    return sub ? a << 1 : a;
}

// svt_ext_all_sad_calculation_8x8_16x16_c (EbMotionEstimation.c:336-368): 8 positions x = 0..7 of a 64x64 block, lane
// = 8x8 block in Z-order; the positions are taken in order so the strict "<" updates match the reference's
__global__ void all_sad_8x8_16x16_kernel(const uint8_t *src, int ss, const uint8_t *ref, int rs, uint32_t mv,
                                         uint32_t *best8, uint32_t *best16, uint32_t *mv8, uint32_t *mv16,
                                         uint32_t *eight16, int sub) {
    const int L = threadIdx.x;
    int       bx, by;
    z8(L, bx, by);
    uint32_t b8 = best8[L], m8 = mv8[L], b16 = best16[L >> 2], m16 = mv16[L >> 2];
    for (int s = 0; s < 8; s++) {
        const uint32_t v8  = sad8x8(src + by * ss + bx, ss, ref + by * rs + bx + s, rs, sub != 0);
        const uint32_t v16 = lane_sum(v8, 1, 4);
        const uint32_t m   = ((uint32_t)(uint16_t)(int16_t)(mv >> 16) << 16) | (uint16_t)((int16_t)(mv & 0xFFFF) + s);
        if (v8 < b8) b8 = v8, m8 = m;
        if (v16 < b16) b16 = v16, m16 = m;
        if ((L & 3) == 0) eight16[(L >> 2) * 8 + s] = v16;
    }
    best8[L] = b8, mv8[L] = m8;
    if ((L & 3) == 0) best16[L >> 2] = b16, mv16[L >> 2] = m16;
}

// svt_ext_eight_sad_calculation_32x32_64x64_c (:370-428) and svt_ext_sad_calculation_32x32_64x64_c (:172-210):
// npos positions (8 or 1) of 16x16 SADs [16][npos] -> 32x32 / 64x64 sums and best updates; lane = position
__global__ void sad_32x32_64x64_kernel(const uint32_t *sad16, int npos, uint32_t *best32, uint32_t *best64,
                                       uint32_t *mv32, uint32_t *mv64, uint32_t mv, uint32_t *sad32) {
    if (threadIdx.x != 0) return; // the strict "<" updates run in position order
    for (int s = 0; s < npos; s++) {
        const uint32_t m = npos == 1 ? mv
                                     : ((uint32_t)(uint16_t)(int16_t)(mv >> 16) << 16) |
                                           (uint16_t)((int16_t)(mv & 0xFFFF) + s);
        uint32_t s64 = 0;
        for (int k = 0; k < 4; k++) {
            uint32_t v = 0;
            for (int j = 0; j < 4; j++) v += sad16[(4 * k + j) * npos + s];
            sad32[k * npos + s] = v;
            if (v < best32[k]) best32[k] = v, mv32[k] = m;
            s64 += v;
        }
        if (s64 < best64[0]) best64[0] = s64, mv64[0] = m;
    }
}

// svt_ext_sad_calculation_8x8_16x16_c (:99-170): one 16x16 block at one position
__global__ void sad_8x8_16x16_kernel(const uint8_t *src, int ss, const uint8_t *ref, int rs, uint32_t *best8,
                                     uint32_t *best16, uint32_t *mv8, uint32_t *mv16, uint32_t mv, uint32_t *sad16,
                                     uint32_t *sad8, int sub) {
    const int k = threadIdx.x;
    uint32_t  v = 0;
    if (k < 4) v = sad8x8(src + 8 * (k >> 1) * ss + 8 * (k & 1), ss, ref + 8 * (k >> 1) * rs + 8 * (k & 1), rs, sub);
    const uint32_t t = lane_sum(v, 1, 4);
    if (k < 4) {
        sad8[k] = v;
        if (v < best8[k]) best8[k] = v, mv8[k] = mv;
    }
    if (k == 0) {
        if (t < best16[0]) best16[0] = t, mv16[0] = mv;
        sad16[0] = t;
    }
}

// svt_sad_loop_kernel_c (EbComputeSAD_C.c:58-99): every (x, y) of the search area, ref advancing by src_stride_raw per
// search row; best = first minimum below 0xffffff in (y, x) order
__global__ __launch_bounds__(256) void sad_loop_kernel(const uint8_t *src, int ss, const uint8_t *ref, int rs, int bh,
                                                       int bw, int srr, int skip_rows, int saw, int sah,
                                                       unsigned long long *out) {
    const int n = saw * sah;
    unsigned long long best = ~0ull; // (sad << 32) | scan index
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const int y = p / saw, x = p - y * saw;
        if (skip_rows && (y & 1) == 0) continue;
        const uint8_t *r = ref + (size_t)y * srr + x;
        uint32_t       a = 0;
        for (int j = 0; j < bh; j++)
            for (int i = 0; i < bw; i++) a += (uint32_t)abs((int)src[j * ss + i] - (int)r[j * rs + i]);
        const unsigned long long key = ((unsigned long long)a << 32) | (uint32_t)p;
        best = key < best ? key : best;
    }
    for (int o = 32; o; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o, 64);
        best = v < best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(out, best);
}

// host staging of a strided host region as one linear device span
struct Span {
    uint8_t *d = nullptr;
    ~Span() { (void)hipFree(d); }
};
void upload_span(hipStream_t st, Span &sp, const uint8_t *h, size_t bytes) {
    HIP_OR_DIE(hipMalloc(&sp.d, bytes ? bytes : 1));
    HIP_OR_DIE(hipMemcpyAsync(sp.d, h, bytes, hipMemcpyHostToDevice, st));
}
template <typename W>
W *upload_words(hipStream_t st, Span &sp, const W *h, size_t n) {
    upload_span(st, sp, (const uint8_t *)h, n * sizeof(W));
    return (W *)sp.d;
}
template <typename W>
void download_words(hipStream_t st, W *h, const Span &sp, size_t n) {
    HIP_OR_DIE(hipMemcpyAsync(h, sp.d, n * sizeof(W), hipMemcpyDeviceToHost, st));
}

} // namespace

struct SvtGpuMeBatch {
    SvtGpuContext *ctx;
    int32_t        width, height, nref, nsbx, nsby;
    int16_t       *d_origin;
    uint32_t      *d_sad, *d_mv;
};

extern "C" int svtgpu_me_batch_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t nref,
                                      SvtGpuMeBatch **out) {
    if (!ctx || !out || width <= 0 || height <= 0 || nref < 1 || nref > 8) return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    SvtGpuMeBatch *b = new SvtGpuMeBatch();
    b->ctx = ctx, b->width = width, b->height = height, b->nref = nref;
    b->nsbx = (width + 63) / 64, b->nsby = (height + 63) / 64;
    const size_t n = (size_t)b->nsbx * b->nsby * nref;
    hipError_t   e = hipMalloc(&b->d_origin, n * 2 * sizeof(int16_t));
    if (e == hipSuccess) e = hipMalloc(&b->d_sad, n * kOut * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&b->d_mv, n * kOut * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(b->d_origin, 0, n * 2 * sizeof(int16_t));
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr); // null-stream memset done before the caller's streams run
    if (e != hipSuccess) {
        svtgpu_me_batch_destroy(b);
        svtgpu_set_last_hip_error(e, "me batch alloc", __FILE__, __LINE__);
        return e == hipErrorOutOfMemory ? SVTGPU_ERR_OOM : SVTGPU_ERR_HIP;
    }
    *out = b;
    return SVTGPU_OK;
}

extern "C" void svtgpu_me_batch_destroy(SvtGpuMeBatch *b) {
    if (!b) return;
    (void)hipFree(b->d_origin);
    (void)hipFree(b->d_sad);
    (void)hipFree(b->d_mv);
    delete b;
}

extern "C" int svtgpu_me_set_origins(SvtGpuMeBatch *b, const int16_t *origin, void *stream) {
    if (!b || !origin) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t  st = pick_stream(b->ctx, stream);
    const size_t n  = (size_t)b->nsbx * b->nsby * b->nref * 2 * sizeof(int16_t);
    HIP_TRY(hipMemcpyAsync(b->d_origin, origin, n, hipMemcpyHostToDevice, st));
    svtgpu_count_xfer(0, n);
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

extern "C" int svtgpu_me_search(SvtGpuMeBatch *b, const SvtGpuFrame *source, const SvtGpuFrame *const *refs,
                                int32_t search_area_width, int32_t search_area_height, int32_t sub_sad,
                                int32_t sb_begin, int32_t sb_end, void *stream) {
    const int nsb = b ? b->nsbx * b->nsby : 0;
    if (!b || !source || !refs || source->width != b->width || source->height != b->height || sb_begin < 0 ||
        sb_end > nsb || sb_begin > sb_end || search_area_width < 1 || search_area_height < 1)
        return SVTGPU_ERR_INVALID_ARG;
    if (source->bit_depth != 8 || search_area_width > kMaxSaw) return SVTGPU_ERR_UNSUPPORTED;
    MeArgs a;
    std::memset(&a, 0, sizeof a);
    a.src = (const uint8_t *)source->plane[0], a.src_stride = source->stride[0];
    a.width = b->width, a.height = b->height, a.nsbx = b->nsbx, a.nref = b->nref, a.sb_begin = sb_begin;
    for (int r = 0; r < b->nref; r++) {
        const SvtGpuFrame *f = refs[r];
        if (!f || f->width != b->width || f->height != b->height || f->bit_depth != 8) return SVTGPU_ERR_INVALID_ARG;
        a.ref[r] = (const uint8_t *)f->plane[0], a.ref_stride[r] = f->stride[0];
    }
    a.origin = b->d_origin, a.saw = search_area_width, a.sah = search_area_height, a.sub = sub_sad != 0;
    a.best_sad = b->d_sad, a.best_mv = b->d_mv;
    if (sb_end == sb_begin) return SVTGPU_OK;
    hipStream_t st = pick_stream(b->ctx, stream);
    hipLaunchKernelGGL(me_search_kernel, dim3((sb_end - sb_begin) * b->nref), dim3(256), 0, st, a);
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

extern "C" int svtgpu_me_read(SvtGpuMeBatch *b, uint32_t *best_sad, uint32_t *best_mv, int32_t sb_begin,
                              int32_t sb_end, void *stream) {
    const int nsb = b ? b->nsbx * b->nsby : 0;
    if (!b || sb_begin < 0 || sb_end > nsb || sb_begin > sb_end) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t  st  = pick_stream(b->ctx, stream);
    const size_t row = (size_t)b->nref * kOut, n = (size_t)(sb_end - sb_begin) * row * sizeof(uint32_t);
    if (best_sad) HIP_TRY(hipMemcpyAsync(best_sad, b->d_sad + sb_begin * row, n, hipMemcpyDeviceToHost, st));
    if (best_mv) HIP_TRY(hipMemcpyAsync(best_mv, b->d_mv + sb_begin * row, n, hipMemcpyDeviceToHost, st));
    svtgpu_count_xfer(1, (best_sad ? n : 0) + (best_mv ? n : 0));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}

// ---- RTCD shims (aom_dsp_rtcd.h:776, 839, 845, 850, 851): synchronous, host pointers ----
extern "C" void svtgpu_ext_all_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref,
                                                         uint32_t ref_stride, uint32_t mv, uint32_t *p_best_sad_8x8,
                                                         uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                                         uint32_t *p_best_mv16x16, uint32_t p_eight_sad16x16[16][8],
                                                         uint32_t p_eight_sad8x8[64][8], Bool sub_sad) {
    (void)p_eight_sad8x8; // not written by the reference's C either (EbMotionEstimation.c:223)
    hipStream_t st = svtgpu_shim_stream();
    Span        s, r, b8, b16, m8, m16, e16;
    upload_span(st, s, src, (size_t)63 * src_stride + 64);
    upload_span(st, r, ref, (size_t)63 * ref_stride + 64 + 7);
    uint32_t *d8 = upload_words(st, b8, p_best_sad_8x8, 64), *d16 = upload_words(st, b16, p_best_sad_16x16, 16);
    uint32_t *dm8 = upload_words(st, m8, p_best_mv8x8, 64), *dm16 = upload_words(st, m16, p_best_mv16x16, 16);
    uint32_t *de = upload_words(st, e16, &p_eight_sad16x16[0][0], 128);
    hipLaunchKernelGGL(all_sad_8x8_16x16_kernel, dim3(1), dim3(64), 0, st, s.d, (int)src_stride, r.d, (int)ref_stride,
                       mv, d8, d16, dm8, dm16, de, (int)sub_sad);
    HIP_OR_DIE(hipGetLastError());
    download_words(st, p_best_sad_8x8, b8, 64), download_words(st, p_best_sad_16x16, b16, 16);
    download_words(st, p_best_mv8x8, m8, 64), download_words(st, p_best_mv16x16, m16, 16);
    download_words(st, &p_eight_sad16x16[0][0], e16, 128);
    HIP_OR_DIE(hipStreamSynchronize(st));
}

static void sad_32_64(const uint32_t *sad16, int npos, uint32_t *best32, uint32_t *best64, uint32_t *mv32,
                      uint32_t *mv64, uint32_t mv, uint32_t *sad32) {
    hipStream_t st = svtgpu_shim_stream();
    Span        a, b32, b64, m32, m64, s32;
    uint32_t   *da = upload_words(st, a, sad16, 16 * (size_t)npos);
    uint32_t   *d32 = upload_words(st, b32, best32, 4), *d64 = upload_words(st, b64, best64, 1);
    uint32_t   *dm32 = upload_words(st, m32, mv32, 4), *dm64 = upload_words(st, m64, mv64, 1);
    uint32_t   *ds = upload_words(st, s32, sad32, 4 * (size_t)npos);
    hipLaunchKernelGGL(sad_32x32_64x64_kernel, dim3(1), dim3(64), 0, st, da, npos, d32, d64, dm32, dm64, mv, ds);
    HIP_OR_DIE(hipGetLastError());
    download_words(st, best32, b32, 4), download_words(st, best64, b64, 1);
    download_words(st, mv32, m32, 4), download_words(st, mv64, m64, 1);
    download_words(st, sad32, s32, 4 * (size_t)npos);
    HIP_OR_DIE(hipStreamSynchronize(st));
}

extern "C" void svtgpu_ext_eight_sad_calculation_32x32_64x64(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                             uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                             uint32_t *p_best_mv64x64, uint32_t mv,
                                                             uint32_t p_sad32x32[4][8]) {
    sad_32_64(&p_sad16x16[0][0], 8, p_best_sad_32x32, p_best_sad_64x64, p_best_mv32x32, p_best_mv64x64, mv,
              &p_sad32x32[0][0]);
}

extern "C" void svtgpu_ext_sad_calculation_32x32_64x64(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                                       uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                       uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32) {
    sad_32_64(p_sad16x16, 1, p_best_sad_32x32, p_best_sad_64x64, p_best_mv32x32, p_best_mv64x64, mv, p_sad32x32);
}

extern "C" void svtgpu_ext_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref,
                                                     uint32_t ref_stride, uint32_t *p_best_sad_8x8,
                                                     uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                                     uint32_t *p_best_mv16x16, uint32_t mv, uint32_t *p_sad16x16,
                                                     uint32_t *p_sad8x8, Bool sub_sad) {
    hipStream_t st = svtgpu_shim_stream();
    Span        s, r, b8, b16, m8, m16, s16, s8;
    upload_span(st, s, src, (size_t)15 * src_stride + 16);
    upload_span(st, r, ref, (size_t)15 * ref_stride + 16);
    uint32_t *d8 = upload_words(st, b8, p_best_sad_8x8, 4), *d16 = upload_words(st, b16, p_best_sad_16x16, 1);
    uint32_t *dm8 = upload_words(st, m8, p_best_mv8x8, 4), *dm16 = upload_words(st, m16, p_best_mv16x16, 1);
    uint32_t *ds16 = upload_words(st, s16, p_sad16x16, 1), *ds8 = upload_words(st, s8, p_sad8x8, 4);
    hipLaunchKernelGGL(sad_8x8_16x16_kernel, dim3(1), dim3(64), 0, st, s.d, (int)src_stride, r.d, (int)ref_stride, d8,
                       d16, dm8, dm16, mv, ds16, ds8, (int)sub_sad);
    HIP_OR_DIE(hipGetLastError());
    download_words(st, p_best_sad_8x8, b8, 4), download_words(st, p_best_sad_16x16, b16, 1);
    download_words(st, p_best_mv8x8, m8, 4), download_words(st, p_best_mv16x16, m16, 1);
    download_words(st, p_sad16x16, s16, 1), download_words(st, p_sad8x8, s8, 4);
    HIP_OR_DIE(hipStreamSynchronize(st));
}

extern "C" void svtgpu_sad_loop_kernel(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                       uint32_t block_height, uint32_t block_width, uint64_t *best_sad,
                                       int16_t *x_search_center, int16_t *y_search_center, uint32_t src_stride_raw,
                                       uint8_t skip_search_line, int16_t search_area_width,
                                       int16_t search_area_height) {
    *best_sad = 0xffffff;
    if (search_area_width <= 0 || search_area_height <= 0 || !block_width || !block_height) return;
    hipStream_t st = svtgpu_shim_stream();
    Span        s, r, o;
    upload_span(st, s, src, (size_t)(block_height - 1) * src_stride + block_width);
    upload_span(st, r, ref,
                (size_t)(search_area_height - 1) * src_stride_raw + (search_area_width - 1) +
                    (size_t)(block_height - 1) * ref_stride + block_width);
    const unsigned long long init = ~0ull;
    unsigned long long      *d    = upload_words(st, o, &init, 1);
    const int skip = block_width == 16 && block_height <= 16 && skip_search_line;
    const int n    = search_area_width * search_area_height;
    hipLaunchKernelGGL(sad_loop_kernel, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, st, s.d, (int)src_stride,
                       r.d, (int)ref_stride, (int)block_height, (int)block_width, (int)src_stride_raw, skip,
                       (int)search_area_width, (int)search_area_height, d);
    HIP_OR_DIE(hipGetLastError());
    unsigned long long best = 0;
    HIP_OR_DIE(hipMemcpyAsync(&best, d, 8, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    const uint32_t sad = (uint32_t)(best >> 32), p = (uint32_t)best;
    if (best != ~0ull && sad < 0xffffffu) { // strict "<" against the 0xffffff start (EbComputeSAD_C.c:88-92)
        *best_sad        = sad;
        *x_search_center = (int16_t)(p % (uint32_t)search_area_width);
        *y_search_center = (int16_t)(p / (uint32_t)search_area_width);
    }
}

// ---- svt_pme_sad_loop_kernel (aom_dsp_rtcd.h:866; C EbProductCodingLoop.c:1801-1852): the MD full-pel refinement,
// cost = SAD + svt_aom_fp_mv_err_cost (mcomp.c:43-68, 771) at every visited position ----
namespace {
// layout of the reference's svt_mv_cost_param (mcomp.h:37-48): the shim reads the caller's struct through this view
struct MvCostView {
    const int16_t *ref_mv; // MV {row, col}
    int16_t        full_ref_mv[2];
    uint8_t        mv_cost_type;
    const int     *mvjcost;
    const int     *mvcost[2];
    int            error_per_bit, early_exit_th, sad_per_bit;
};
struct PmeArgs {
    const uint8_t *src, *ref;
    int            ss, rs, bh, bw, npos;
    const int32_t *pos;                  // [npos] (x, y) search indices packed x | y << 16, in the reference's order
    int            start_x, start_y, mvx, mvy, ref_row, ref_col, type, epb;
    const int     *jc;                   // mvjcost[4]
    const int     *rc, *cc;              // mvcost[0][row_lo ..], mvcost[1][col_lo ..] (clipped index ranges)
    int            row_lo, col_lo;
};

__device__ inline int pme_mv_cost(const PmeArgs &a, int row, int col) { // svt_mv_err_cost (mcomp.c:43-68)
    const int dr = row - a.ref_row, dc = col - a.ref_col, ar = abs(dr), ac = abs(dc);
    switch (a.type) {
    case 0: { // MV_COST_ENTROPY: joint + components, clipped to [MV_LOW, MV_UPP]
        if (!a.rc) return 0;
        const int j = dr == 0 ? (dc == 0 ? 0 : 1) : (dc == 0 ? 2 : 3);
        const int r = min(max(dr, -(1 << 14)), 1 << 14), c = min(max(dc, -(1 << 14)), 1 << 14);
        const long long bits = (long long)a.jc[j] + a.rc[r - a.row_lo] + a.cc[c - a.col_lo];
        return (int)((bits * a.epb + (1ll << 13)) >> 14); // RDDIV_BITS + AV1_PROB_COST_SHIFT - RD_EPB_SHIFT + 4
    }
    case 1: return (2 * (ar + ac)) >> 3; // SSE_LAMBDA_LOWRES
    case 2: return 0;                    // SSE_LAMBDA_MIDRES = 0
    case 3: return (ar + ac) >> 3;       // SSE_LAMBDA_HDRES
    case 4: return (int)(((long long)((ar + ac) << 8) * a.epb + (1ll << 13)) >> 14); // MV_COST_OPT
    default: return 0;
    }
}

__global__ __launch_bounds__(256) void pme_kernel(const PmeArgs a, unsigned long long *out) {
    unsigned long long best = ~0ull; // (cost << 32) | order
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < a.npos; p += gridDim.x * blockDim.x) {
        const int xi = a.pos[p] & 0xFFFF, yi = a.pos[p] >> 16;
        const uint8_t *r = a.ref + (size_t)yi * a.rs + xi;
        uint32_t       s = 0;
        for (int y = 0; y < a.bh; y++)
            for (int x = 0; x < a.bw; x++) s += (uint32_t)abs((int)a.src[y * a.ss + x] - (int)r[y * a.rs + x]);
        const int16_t col = (int16_t)(a.mvx + (int)(uint32_t)(a.start_x + xi) * 8);
        const int16_t row = (int16_t)(a.mvy + (int)(uint32_t)(a.start_y + yi) * 8);
        const uint32_t cost = s + (uint32_t)pme_mv_cost(a, row, col);
        const unsigned long long key = ((unsigned long long)cost << 32) | (uint32_t)p;
        best = key < best ? key : best;
    }
    for (int o = 32; o; o >>= 1) {
        const unsigned long long v = __shfl_xor(best, o, 64);
        best = v < best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(out, best);
}
} // namespace

extern "C" void svtgpu_pme_sad_loop_kernel(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src,
                                           uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                           uint32_t block_height, uint32_t block_width, uint32_t *best_cost,
                                           int16_t *best_mvx, int16_t *best_mvy, int16_t search_position_start_x,
                                           int16_t search_position_start_y, int16_t search_area_width,
                                           int16_t search_area_height, int16_t search_step, int16_t mvx, int16_t mvy) {
    const MvCostView *mc = (const MvCostView *)mv_cost_params;
    // the visited positions in the reference's order (EbProductCodingLoop.c:1812-1826): groups of 8 columns, then a
    // jump of search_step; a group is not started when fewer than 8 columns remain.  col_num and the column step
    // carry over from one search row to the next, as there
    std::vector<int32_t> pos;
    int maxx = 0, maxy = 0, col_num = 0, step_x = 1;
    for (int y = 0; y < search_area_height; y += search_step) {
        for (int x = 0; x < search_area_width; x += step_x) {
            if (search_area_width - x < 8 && col_num == 0) continue;
            if (col_num == 7) col_num = 0, step_x = search_step;
            else col_num++, step_x = 1;
            pos.push_back(x | (y << 16));
            maxx = std::max(maxx, x), maxy = std::max(maxy, y);
        }
    }
    if (pos.empty()) return;
    hipStream_t st = svtgpu_shim_stream();
    PmeArgs     a;
    std::memset(&a, 0, sizeof a);
    a.ss = (int)src_stride, a.rs = (int)ref_stride, a.bh = (int)block_height, a.bw = (int)block_width;
    a.npos = (int)pos.size(), a.start_x = search_position_start_x, a.start_y = search_position_start_y;
    a.mvx = mvx, a.mvy = mvy, a.ref_row = mc->ref_mv[0], a.ref_col = mc->ref_mv[1], a.type = mc->mv_cost_type;
    a.epb = mc->error_per_bit;
    Span s, r, p, o, jc, rc, cc;
    upload_span(st, s, src, (size_t)(block_height - 1) * src_stride + block_width);
    upload_span(st, r, ref, (size_t)(maxy + block_height - 1) * ref_stride + maxx + block_width);
    a.src = s.d, a.ref = r.d;
    a.pos = upload_words(st, p, pos.data(), pos.size());
    if (a.type == 0 && mc->mvcost[0] && mc->mvcost[1] && mc->mvjcost) {
        // the clipped component indices the positions can reach
        auto clip = [](int v) { return std::min(std::max(v, -(1 << 14)), 1 << 14); };
        int rlo = INT32_MAX, rhi = INT32_MIN, clo = INT32_MAX, chi = INT32_MIN;
        for (int32_t q : pos) {
            const int16_t col = (int16_t)(mvx + (int)(uint32_t)(search_position_start_x + (q & 0xFFFF)) * 8);
            const int16_t row = (int16_t)(mvy + (int)(uint32_t)(search_position_start_y + (q >> 16)) * 8);
            const int     rr = clip(row - a.ref_row), cc2 = clip(col - a.ref_col);
            rlo = std::min(rlo, rr), rhi = std::max(rhi, rr), clo = std::min(clo, cc2), chi = std::max(chi, cc2);
        }
        a.row_lo = rlo, a.col_lo = clo;
        a.jc = upload_words(st, jc, mc->mvjcost, 4);
        a.rc = upload_words(st, rc, mc->mvcost[0] + rlo, (size_t)(rhi - rlo + 1));
        a.cc = upload_words(st, cc, mc->mvcost[1] + clo, (size_t)(chi - clo + 1));
    }
    const unsigned long long init = ~0ull;
    unsigned long long      *d    = upload_words(st, o, &init, 1);
    hipLaunchKernelGGL(pme_kernel, dim3(std::min(256, (a.npos + 255) / 256)), dim3(256), 0, st, a, d);
    HIP_OR_DIE(hipGetLastError());
    unsigned long long best = 0;
    HIP_OR_DIE(hipMemcpyAsync(&best, d, 8, hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
    const uint32_t cost = (uint32_t)(best >> 32), q = (uint32_t)pos[(uint32_t)best];
    if (cost < *best_cost) { // strict "<" against the caller's running best, first position in order on ties
        *best_cost = cost;
        *best_mvx  = (int16_t)(mvx + (int)(uint32_t)(search_position_start_x + (int)(q & 0xFFFF)) * 8);
        *best_mvy  = (int16_t)(mvy + (int)(uint32_t)(search_position_start_y + (int)(q >> 16)) * 8);
    }
}
