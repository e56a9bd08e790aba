// cdef_pick.hip — frame-level CDEF strength selection on the device.
//
// ≙ finish_cdef_search (Source/Lib/Encoder/Codec/EbEncCdef.c:728-926).  The expensive part is the
// 75 calls of svt_search_one_dual (:627-695): tot[j][k] = sum_fb min(best_fb, mse0[fb][j] +
// mse1[fb][k]) over 64x64 strength pairs, then the first minimum.  The four greedy chains
// (nb = 1, 2, 4, 8 → 5, 10, 20, 40 dependent calls, :697-727) are independent, so each device step
// advances every chain that is still running: step = one partial-sum kernel (FB chunks x chains)
// + one reduce/argmin kernel per chain that also appends the pick and pre-shifts the selection list
// for the next refinement call.  40 steps, all enqueued without host synchronisation.  The RD
// choice over nb (:853-872) and the filter_map remap (:911-919) are a few scalar ops on the host.
#include <algorithm>
#include <cstring>

#include "svtgpu_internal.h"

#define NT 256
#define MAX_CHAINS 4
#define FB_BATCH 8

struct StepChain {
    int32_t chain;     // 0..3 (nb = 1 << chain)
    int32_t nb_sel;    // number of already-selected pairs for this call
    int32_t shift_after;
    int32_t nb;
};
struct StepArgs {
    const uint64_t *wmse; // [sb_count][2][64] compacted, bias applied
    int32_t         sb_count, chunk, parts, start_gi, end_gi;
    int32_t        *lev;  // [4][2][16]
    uint64_t       *part; // [4][parts][4096]
    uint64_t       *best; // [4]
    StepChain       ch[MAX_CHAINS];
};

// ---- compaction: non-skipped FBs in raster order, zero-strength bias (EbEncCdef.c:820-851) ----
__global__ void pick_compact_kernel(const uint8_t *skip, int nfb, int32_t *fb_list, int32_t *count) {
    __shared__ int32_t base;
    __shared__ int32_t wsum[NT / 64];
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nfb; c0 += NT) {
        const int  fb   = c0 + threadIdx.x;
        const int  keep = fb < nfb && !skip[fb];
        const unsigned long long bal = __ballot(keep);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const int pre  = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int i = 0; i < w; i++) off += wsum[i];
        if (keep) fb_list[off + pre] = fb;
        __syncthreads();
        if (threadIdx.x == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = base;
}

__global__ void pick_gather_kernel(const uint64_t *mse, int nfb, const int32_t *fb_list, const int32_t *count,
                                   int bias, uint64_t *wmse) {
    const int i = blockIdx.x;
    if (i >= *count) return;
    const int fb = fb_list[i];
    const int p = threadIdx.x >> 6, g = threadIdx.x & 63; // 128 threads
    uint64_t  v = mse[((size_t)p * nfb + fb) * 64 + g];
    if (bias && g == 0) v = ((uint64_t)bias * v) >> 6;
    wmse[((size_t)i * 2 + p) * 64 + g] = v;
}

// ---- one svt_search_one_dual call per active chain, partial over an FB chunk ----
__global__ void __launch_bounds__(NT) sod_partial_kernel(const StepArgs A) {
    __shared__ uint64_t m[FB_BATCH][2][64];
    __shared__ int32_t  sel[2][16];
    const StepChain C = A.ch[blockIdx.y];
    const int       t = threadIdx.x, j = t >> 2, k0 = (t & 3) * 16;
    if (t < 32) sel[t >> 4][t & 15] = A.lev[(C.chain * 2 + (t >> 4)) * 16 + (t & 15)];
    uint64_t tot[16];
#pragma unroll
    for (int u = 0; u < 16; u++) tot[u] = 0;
    const int f0 = blockIdx.x * A.chunk, f1 = min(A.sb_count, f0 + A.chunk);
    for (int fb = f0; fb < f1; fb += FB_BATCH) {
        const int nb = min(FB_BATCH, f1 - fb);
        __syncthreads();
        for (int i = t; i < nb * 128; i += NT) (&m[0][0][0])[i] = A.wmse[(size_t)fb * 128 + i];
        __syncthreads();
        for (int b = 0; b < nb; b++) {
            uint64_t best = (uint64_t)1 << 63;
            for (int g = 0; g < C.nb_sel; g++) {
                const uint64_t c = m[b][0][sel[0][g]] + m[b][1][sel[1][g]];
                best = c < best ? c : best;
            }
            const uint64_t mj = m[b][0][j];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const uint64_t c = mj + m[b][1][k0 + u];
                tot[u] += c < best ? c : best;
            }
        }
    }
    uint64_t *out = A.part + ((size_t)C.chain * A.parts + blockIdx.x) * 4096;
#pragma unroll
    for (int u = 0; u < 16; u++) out[j * 64 + k0 + u] = tot[u];
}

// ---- sum partials, first argmin over [start, end)^2, append the pick, pre-shift for refinement ----
__global__ void __launch_bounds__(NT) sod_reduce_kernel(const StepArgs A) {
    __shared__ uint64_t bv[NT];
    __shared__ int32_t  bi[NT];
    const StepChain C = A.ch[blockIdx.x];
    const int       t = threadIdx.x;
    uint64_t        best = (uint64_t)1 << 63; // best_tot_mse initial value (EbEncCdef.c:632)
    int             bidx = 1 << 30;
    for (int u = 0; u < 16; u++) {
        const int e = t * 16 + u, j = e >> 6, k = e & 63;
        uint64_t  s = 0;
        for (int p = 0; p < A.parts; p++) s += A.part[((size_t)C.chain * A.parts + p) * 4096 + e];
        if (j >= A.start_gi && j < A.end_gi && k >= A.start_gi && k < A.end_gi && s < best) {
            best = s;
            bidx = e;
        }
    }
    bv[t] = best;
    bi[t] = bidx;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if (t < w) {
            const uint64_t ov = bv[t + w];
            const int      oi = bi[t + w];
            if (ov < bv[t] || (ov == bv[t] && oi < bi[t])) {
                bv[t] = ov;
                bi[t] = oi;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        int32_t  *l0 = A.lev + C.chain * 32, *l1 = l0 + 16;
        // a search with no candidate returns (1<<63, 0, 0) like the reference's initial values
        const bool any = bi[0] < (1 << 30);
        l0[C.nb_sel] = any ? bi[0] >> 6 : 0;
        l1[C.nb_sel] = any ? bi[0] & 63 : 0;
        A.best[C.chain] = any ? bv[0] : ((uint64_t)1 << 63);
        if (C.shift_after)
            for (int q = 0; q < C.nb - 1; q++) {
                l0[q] = l0[q + 1];
                l1[q] = l1[q + 1];
            }
    }
}

// ---- per-FB strength index (EbEncCdef.c:866-890) ----
__global__ void pick_assign_kernel(const uint64_t *wmse, const int32_t *fb_list, const int32_t *count, int nb,
                                   const int32_t *ygi, int8_t *fb_strength) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const uint64_t *m0 = wmse + (size_t)i * 128, *m1 = m0 + 64;
    uint64_t        best = (uint64_t)1 << 63;
    int             bg   = 0;
    for (int g = 0; g < nb; g++) {
        const uint64_t c = m0[ygi[g]] + m1[ygi[16 + g]];
        if (c < best) {
            best = c;
            bg   = g;
        }
    }
    fb_strength[fb_list[i]] = (int8_t)bg;
}

int svtgpu_cdef_pick_impl(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                          uint64_t lambda, SvtGpuCdefParams *params, int8_t *fb_strength_out, hipStream_t st) {
    const int nfb = s->nfb;
    const int end = ctrls->first_pass_fs_num + ctrls->default_second_pass_fs_num;
    if (end <= 0 || end > 64)
        return SVTGPU_ERR_INVALID_ARG;
    uint64_t *wmse = s->d_pick_part; // layout: [nfb*128] wmse, then partials
    const size_t wmse_elems = (size_t)nfb * 128;
    int32_t  *d_count = s->d_fb_list + nfb;
    hipLaunchKernelGGL(pick_compact_kernel, dim3(1), dim3(NT), 0, st, s->d_skip, nfb, s->d_fb_list, d_count);
    hipLaunchKernelGGL(pick_gather_kernel, dim3(nfb), dim3(128), 0, st, s->d_mse, nfb, s->d_fb_list, d_count,
                       (int)ctrls->zero_fs_cost_bias, wmse);
    int32_t sb_count = 0;
    HIP_TRY(hipMemcpyAsync(&sb_count, d_count, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));

    StepArgs A;
    A.wmse     = wmse;
    A.sb_count = sb_count;
    A.parts    = std::max(1, std::min(s->pick_parts, (sb_count + 63) / 64));
    A.chunk    = (sb_count + A.parts - 1) / A.parts;
    if (A.chunk == 0) A.chunk = 1;
    A.start_gi = 0;
    A.end_gi   = end;
    A.lev      = s->d_pick_lev;
    A.part     = wmse + wmse_elems;
    A.best     = s->d_pick_out;
    HIP_TRY(hipMemsetAsync(s->d_pick_lev, 0, sizeof(int32_t) * MAX_CHAINS * 32, st));
    for (int step = 0; step < 40; step++) {
        int na = 0;
        for (int c = 0; c < MAX_CHAINS; c++) {
            const int nb = 1 << c, len = 5 * nb;
            if (step >= len) continue;
            StepChain &C  = A.ch[na++];
            C.chain       = c;
            C.nb          = nb;
            C.nb_sel      = step < nb ? step : nb - 1;
            C.shift_after = (step + 1 < len) && (step + 1 >= nb);
        }
        hipLaunchKernelGGL(sod_partial_kernel, dim3(A.parts, na), dim3(NT), 0, st, A);
        hipLaunchKernelGGL(sod_reduce_kernel, dim3(na), dim3(NT), 0, st, A);
    }
    HIP_TRY(hipGetLastError());
    int32_t  lev[MAX_CHAINS][2][16];
    uint64_t best[MAX_CHAINS];
    HIP_TRY(hipMemcpyAsync(lev, s->d_pick_lev, sizeof lev, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(best, s->d_pick_out, sizeof best, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));

    // RD choice over the number of signalled strengths (EbEncCdef.c:853-872)
    memset(params, 0, sizeof(*params));
    uint64_t best_cost = (uint64_t)1 << 63;
    int      nbits     = 0;
    for (int i = 0; i <= 3; i++) {
        const int      nb   = 1 << i;
        const int      bits = sb_count * i + nb * 6 * 2;
        const int64_t  rate = (int64_t)bits << 9;                              // av1_cost_literal
        const uint64_t cost = (uint64_t)(((rate * (int64_t)lambda + 256) >> 9) + ((int64_t)(best[i] * 16) << 7)); // RDCOST
        if (cost < best_cost) {
            best_cost = cost;
            nbits     = i;
            for (int j = 0; j < nb; j++) {
                params->cdef_y_strength[j]  = (uint8_t)lev[i][0][j];
                params->cdef_uv_strength[j] = (uint8_t)lev[i][1][j];
            }
        }
    }
    const int nb      = 1 << nbits;
    params->cdef_bits = (uint8_t)nbits;
    int32_t gis[32];
    for (int j = 0; j < 16; j++) {
        gis[j]      = params->cdef_y_strength[j];
        gis[16 + j] = params->cdef_uv_strength[j];
    }
    int32_t *d_gis = s->d_pick_lev + MAX_CHAINS * 32;
    HIP_TRY(hipMemcpyAsync(d_gis, gis, sizeof gis, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(s->d_fb_strength, 0, nfb, st));
    hipLaunchKernelGGL(pick_assign_kernel, dim3((nfb + NT - 1) / NT), dim3(NT), 0, st, wmse, s->d_fb_list, d_count, nb,
                       d_gis, s->d_fb_strength);
    HIP_TRY(hipGetLastError());
    if (fb_strength_out) {
        HIP_TRY(hipMemcpyAsync(fb_strength_out, s->d_fb_strength, nfb, hipMemcpyDeviceToHost, st));
    }
    // gi -> strength code (filter_map, EbEncCdef.c:911-919); damping (:921)
    const int nf = ctrls->first_pass_fs_num;
    for (int i = 0; i < nb; i++) {
        const int y = params->cdef_y_strength[i], uv = params->cdef_uv_strength[i];
        params->cdef_y_strength[i]  = y < nf ? ctrls->default_first_pass_fs[y] : ctrls->default_second_pass_fs[y - nf];
        params->cdef_uv_strength[i] = uv < nf ? ctrls->default_first_pass_fs[uv] : ctrls->default_second_pass_fs[uv - nf];
    }
    params->cdef_damping = (uint8_t)(3 + (base_q_idx >> 6));
    HIP_TRY(hipStreamSynchronize(st));
    return SVTGPU_OK;
}
