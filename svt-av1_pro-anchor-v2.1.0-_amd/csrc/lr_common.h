// lr_common.h — device tables and per-pixel helpers shared by the loop-restoration apply (lr.hip) and
// search (lr_search.hip) kernels.  Reference: Source/Lib/Common/Codec/EbRestoration.c:49-103, 647-760.
#pragma once
#include "svtgpu_internal.h"

#include <vector>

struct SvtGpuLrState {
    SvtGpuContext  *ctx;
    int32_t         width, height;
    int32_t         unit_size[3], hunits[3], vunits[3];
    SvtGpuRestUnit *d_units[3]; // one allocation, planes in order (the search uploads all three in one copy)
    // search scratch (allocated on the first svtgpu_lr_search_frame)
    int16_t        *d_flt;   // per plane [eps][2][W*H] self-guided filter outputs of every searched ep
    size_t          flt_bytes;
    void           *d_work;  // per-unit / per-tile accumulators, descents, work lists
    size_t          work_bytes;
    void           *h_pin;   // pinned host staging for the search's read-backs
    size_t          pin_bytes;
    void           *prof;    // per-kernel-class timing of the search (svtgpu_lr_profile), nullptr when off
    // the tile/unit plan last uploaded into d_work (re-sent only when it changes or d_work moves)
    void                *plan_work;
    std::vector<uint8_t> plan_bytes;
    hipEvent_t           pin_free; // the last copy out of h_pin has run: the host may rewrite it
    hipStream_t          wst;      // the search's Wiener chain (the caller's stream carries the self-guided one)
    hipEvent_t           ev_fork, ev_join;
    // uncached device memory: the exchange words of the resident descents' row parts (coherent without cache flushes)
    void                *d_qarena;
    size_t               qarena_bytes;
    // cached device memory for the self-guided row parts' exchange when it stays in one XCD's L2 (SVTGPU_SR_XCH=l2),
    // and the search count that tags its words (a line left in an L2 by an earlier search never matches a tag)
    void                *d_sxarena;
    size_t               sxarena_bytes;
    uint32_t             sx_epoch;
    // a picture tiled over GPUs (svtgpu_lr_set_tile): the units searched {col0, row0, col1, row1} and the samples
    // written {x0, y0, x1, y1} per plane, the exchange of the search records (null: one rank)
    int32_t              tile_units[3][4], tile_out[3][4];
    SvtGpuComm          *comm;
    // the device RD finish (round 6): its result words in mapped pinned memory, the sequence number of the last finish
    // queued, whether its result has not been collected yet (svtgpu_lr_read_result), the last frame types collected
    int32_t             *h_fout, *h_fout_dev;
    int32_t              fin_seq, fin_pending;
    int32_t              last_ft[3];
};
void lr_profiler_destroy(void *prof);
int  lr_make_wiener_stream(SvtGpuLrState *s); // the search's Wiener-chain stream and its fork / join events
// The restored area of a plane: the frame's crop size (frm_size.frame_width / _height; chroma rounded up, the
// reference's crop_widths / crop_heights, EbPictureBufferDesc.c) -- the device frames themselves are the 8-aligned
// coded size the deblocking and CDEF stages cover (mi_cols x 4)
inline int lr_plane_w(const SvtGpuLrState *s, int p) { return p ? (s->width + 1) >> 1 : s->width; }
inline int lr_plane_h(const SvtGpuLrState *s, int p) { return p ? (s->height + 1) >> 1 : s->height; }
inline bool lr_frame_fits(const SvtGpuLrState *s, const SvtGpuFrame *f) {
    return f && f->width == ((s->width + 7) & ~7) && f->height == ((s->height + 7) & ~7);
}

namespace {

constexpr int NTHR = 256;
// self-guided parameter sets svt_aom_eb_sgr_params (EbRestoration.c:85-103): radii and s values
__constant__ int c_sgr_r[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                                   {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};
__constant__ int c_sgr_s[16][2] = {{140, 3236}, {112, 2158}, {93, 1618}, {80, 1438}, {70, 1295}, {58, 1177},
                                   {47, 1079},  {37, 996},   {30, 925},  {25, 863},  {-1, 2589}, {-1, 1618},
                                   {-1, 1177},  {-1, 925},   {56, -1},   {22, -1}};
// svt_aom_eb_x_by_xplus1 (EbRestoration.c:647-662): round(256 x / (x + 1)), 0 -> 1, 255 -> 256
__constant__ int c_x_by_xplus1[256] = {
    1,   128, 171, 192, 205, 213, 219, 224, 228, 230, 233, 235, 236, 238, 239, 240, 241, 242, 243, 243, 244, 244,
    245, 245, 246, 246, 247, 247, 247, 247, 248, 248, 248, 248, 249, 249, 249, 249, 249, 250, 250, 250, 250, 250,
    250, 250, 251, 251, 251, 251, 251, 251, 251, 251, 251, 251, 252, 252, 252, 252, 252, 252, 252, 252, 252, 252,
    252, 252, 252, 252, 252, 252, 252, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253,
    253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 256};
// svt_aom_eb_one_by_x (EbRestoration.c:664-667): round(4096 / n)
__constant__ int c_one_by_x[25] = {4096, 2048, 1365, 1024, 819, 683, 585, 512, 455, 410, 372, 341, 315,
                                   293,  273,  256,  241,  228, 216, 205, 195, 186, 178, 171, 164};

struct WienerRound {
    int r0, r1;
};
// get_conv_params_wiener (EbRestoration.c:49-72)
__host__ __device__ inline WienerRound wiener_round(int bd) {
    WienerRound r{3, 11};
    const int   over = bd + 7 - 3 + 2 - 16;
    if (over > 0) r.r0 += over, r.r1 -= over;
    return r;
}

// ---------------------------------------------------------------------------------------------
// tile filters over an LDS image `v` (u16, row stride vs) whose (0,0) is the tile's first output
// ---------------------------------------------------------------------------------------------
// Wiener: horizontal 8-tap pass into t (rows -3..h+3 -> t rows 0..h+6), vertical pass into out.
// i / d for 0 <= i < 2^25, 1 <= d <= 128 by one 64-bit multiply: m = ceil(2^32 / d) (exact in that range: the
// error i * (m - 2^32 / d) / 2^32 stays below the distance 1/d to the next integer)
struct FastDiv {
    uint64_t m;
    __device__ explicit FastDiv(uint32_t d) : m(0xFFFFFFFFull / d + 1) {}
    __device__ int operator()(int i) const { return (int)(((uint64_t)(uint32_t)i * m) >> 32); }
};

typedef short v2i16lr __attribute__((ext_vector_type(2)));

template <typename T>
__device__ void wiener_tile(const uint16_t *v, int vs, uint16_t *t, int ts, int w, int h, const int16_t *fx,
                            const int16_t *fy, int bd, T *out, size_t os) {
    const WienerRound rr  = wiener_round(bd);
    const int         lim = (1 << (bd + 1 + 7 - rr.r0)) - 1;
    const FastDiv     dw(w);
    int16_t           vy[8];
    // horizontal taps as int16 pairs for v_dot2, the add-source term folded into the centre tap (|tap3 + 128| fits)
    uint32_t          hp[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        hp[k] = (uint32_t)(uint16_t)(fx[2 * k] + (2 * k == 3 ? 128 : 0)) |
                ((uint32_t)(uint16_t)(fx[2 * k + 1] + (2 * k + 1 == 3 ? 128 : 0)) << 16);
#pragma unroll
    for (int k = 0; k < 8; k++) vy[k] = fy[k];
    // the 8 samples x-3 .. x+4 of a row from 5 aligned dwords and funnel shifts (`v` is 4-byte aligned): adjacent
    // 16-bit reads merged by the compiler would be misaligned for half the lanes, far below the LDS rate
    const uint32_t *vw = (const uint32_t *)v;
    for (int i = threadIdx.x; i < (h + 7) * w; i += NTHR) {
        const int       q = dw(i), y = q - 3, x = i - q * w;
        const int       a = y * vs + x - 3, sh = (a & 1) * 16;
        const uint32_t *wp = vw + (a >> 1);
        uint32_t        wd[5];
#pragma unroll
        for (int k = 0; k < 5; k++) wd[k] = wp[k];
        int sum = 1 << (bd + 6);
#pragma unroll
        for (int k = 0; k < 4; k++)
            sum = __builtin_amdgcn_sdot2(__builtin_bit_cast(v2i16lr, __builtin_amdgcn_alignbit(wd[k + 1], wd[k], sh)),
                                         __builtin_bit_cast(v2i16lr, hp[k]), sum, false);
        t[(y + 3) * ts + x] = (uint16_t)min(max((sum + (1 << (rr.r0 - 1))) >> rr.r0, 0), lim);
    }
    __syncthreads();
    const int maxv = (1 << bd) - 1;
    for (int i = threadIdx.x; i < h * w; i += NTHR) {
        const int       y = dw(i), x = i - y * w;
        const uint16_t *c = t + y * ts + x; // rows y-3 .. y+4 of the intermediate
        int             sum = ((int)c[3 * ts] << 7) - (1 << (bd + rr.r1 - 1));
#pragma unroll
        for (int k = 0; k < 8; k++) sum += (int)c[k * ts] * vy[k];
        out[y * os + x] = (T)min(max((sum + (1 << (rr.r1 - 1))) >> rr.r1, 0), maxv);
    }
}

// A, B of a self-guided pass from the box sum / sum of squares over n = (2r+1)^2 pixels
// (selfguided_restoration_*_internal, EbRestoration.c:693-760); u32 arithmetic wraps like the reference's
__device__ inline void sgr_ab_from_sums(int sum, int sq, int n, int s, int bd, const int *x_by_xplus1, int *A,
                                        int *B) {
    const uint32_t a = (uint32_t)((sq + ((1 << (2 * (bd - 8))) >> 1)) >> (2 * (bd - 8)));
    const uint32_t b = (uint32_t)((sum + ((1 << (bd - 8)) >> 1)) >> (bd - 8));
    const uint32_t p = (a * n < b * b) ? 0u : a * n - b * b;
    const uint32_t z = (p * (uint32_t)s + (1u << 19)) >> 20;
    *A               = x_by_xplus1[min(z, 255u)];
    *B = (int)(((uint32_t)(256 - *A) * (uint32_t)sum * (uint32_t)c_one_by_x[n - 1] + (1u << 11)) >> 12);
}

// A, B of one self-guided pass at (i, j) of an LDS image
__device__ inline void sgr_ab(const uint16_t *v, int vs, int i, int j, int r, int s, int bd, int *A, int *B) {
    int sum = 0, sq = 0;
    for (int y = -r; y <= r; y++)
        for (int x = -r; x <= r; x++) {
            const int p = v[(i + y) * vs + j + x];
            sum += p;
            sq += p * p;
        }
    sgr_ab_from_sums(sum, sq, (2 * r + 1) * (2 * r + 1), s, bd, c_x_by_xplus1, A, B);
}

} // namespace
