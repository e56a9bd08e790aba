// cdef_pick.hip — frame-level CDEF strength selection on the device.
//
// ≙ finish_cdef_search (Source/Lib/Encoder/Codec/EbEncCdef.c:728-926).  The expensive part is the
// 75 calls of svt_search_one_dual (:627-695): tot[j][k] = sum_fb min(best_fb, mse0[fb][j] +
// mse1[fb][k]) over 64x64 strength pairs, then the first minimum.  The four greedy chains
// (nb = 1, 2, 4, 8 → 5, 10, 20, 40 dependent calls, :697-727) are independent, so each device step
// advances every chain that is still running: step = one partial-sum kernel (FB chunks x chains)
// + one reduce/argmin kernel per chain that also appends the pick and pre-shifts the selection list
// for the next refinement call.  40 steps, all enqueued without host synchronisation (the grid is shaped
// for every FB; workgroups past the non-skipped count read on the device find no work).  The RD choice over
// nb (:853-872) and the per-FB assignment run on the device too and write the result straight into mapped
// pinned memory: one host synchronisation per pick.  The filter_map remap (:911-919) stays on the host.
#include <algorithm>
#include <cstring>

#include "svtgpu_internal.h"

#define NT 256
#define MAX_CHAINS 4
#define NSTEPS 40            // longest chain: nb = 8 → 8 + 32 calls (EbEncCdef.c:714-726)
#define PICK_CHUNK 48        // max FBs per workgroup (staged in LDS: <= 48.4 KB; a multiple of 4)

struct StepChain {
    int32_t chain;       // 0..3 (nb = 1 << chain)
    int32_t nb;
    int32_t nb_sel;      // selection size of this call (-1: finalize only)
    int32_t prev_nb_sel; // selection size of the previous call (-1: none)
    int32_t prev_shift;  // the previous call's result is followed by a refinement shift
};
struct StepArgs {
    const uint64_t *wmse;   // [sb_count][2][64] compacted, bias applied
    const int32_t  *count;  // sb_count, the number of non-skipped FBs (device)
    const int32_t  *wide;   // nonzero when some wmse entry is >= 2^31 (the 32-bit path would not be exact)
    int32_t         chunk, start_gi, end_gi, step, na; // na: chains in this launch
    int32_t         fb_alloc;                           // FB rows the wmse table holds
    uint64_t       *tot;    // [3][4][4096] rotating tot_mse accumulators
    int32_t        *lev;    // [NSTEPS+1][4][32] selection list entering each call
    int32_t        *fin;    // [4][32] final list per chain
    uint64_t       *best;   // [4] value returned by each chain's last call
    StepChain       ch[MAX_CHAINS];
    unsigned long long *wgclk; // diagnostics or null
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
                                   int bias, uint64_t *wmse, int32_t *wide) {
    const int i = blockIdx.x;
    if (i >= *count) return;
    const int fb = fb_list[i];
    const int p = threadIdx.x >> 6, g = threadIdx.x & 63; // 128 threads
    uint64_t  v = mse[((size_t)p * nfb + fb) * 64 + g];
    if (bias && g == 0) v = ((uint64_t)bias * v) >> 6;
    wmse[((size_t)i * 2 + p) * 64 + g] = v;
    if (__any(v >> 31)) // m0 + m1 may leave 32 bits: the step kernels keep the 64-bit arithmetic
        if ((threadIdx.x & 63) == 0) atomicOr(wide, 1);
}

// First minimum of tot over [start, end)^2 (svt_search_one_dual's final loop, EbEncCdef.c:670-679),
// computed by every workgroup that needs it from the lane's 16 entries tv[u] = tot[u * NT + t] (loaded by the caller
// at the top of the step).  Returns (best, e = j*64 + k) through LDS.
__device__ __forceinline__ void tot_argmin(const uint64_t (&tv)[4096 / NT], int start, int end, uint64_t *bv, int32_t *bi) {
    const int t    = threadIdx.x;
    uint64_t  best = (uint64_t)1 << 63; // best_tot_mse initial value (EbEncCdef.c:632)
    int       idx  = 1 << 30;
#pragma unroll
    for (int u = 0; u < 4096 / NT; u++) { // ascending e per lane keeps the first minimum
        const int      e = u * NT + t, j = e >> 6, k = e & 63;
        const uint64_t v = tv[u];
        if (j >= start && j < end && k >= start && k < end && v < best) {
            best = v;
            idx  = e;
        }
    }
    // (value, index) minimum over the wave with cross-lane shuffles, then over the 4 waves: 2 barriers instead of 8
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t ov = __shfl_xor(best, o);
        const int      oi = __shfl_xor(idx, o);
        if (ov < best || (ov == best && oi < idx)) best = ov, idx = oi;
    }
    if ((t & 63) == 0) bv[t >> 6] = best, bi[t >> 6] = idx;
    __syncthreads();
    if (t == 0)
        for (int w = 1; w < NT / 64; w++)
            if (bv[w] < bv[0] || (bv[w] == bv[0] && bi[w] < bi[0])) bv[0] = bv[w], bi[0] = bi[w];
    __syncthreads();
}

// One launch per greedy step: every active chain finishes its previous svt_search_one_dual call
// (argmin of the previous tot), forms the selection entering this call (append + refinement shift,
// EbEncCdef.c:714-726) and accumulates this call's tot[j][k] = sum_fb min(best_fb, m0[j] + m1[k]).
// grid (4 tiles of 16 rows j, FB chunks, chains).  The chunk's mse rows are staged in LDS; lane
// k = t & 63, wave q owns rows 16*tile + 4*q + {0..3}; partials meet through u64 atomics.
__global__ void __launch_bounds__(NT) sod_step_kernel(const StepArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn[]; // [chunk][128] mse rows + [chunk] best
    uint64_t (*m)[128] = (uint64_t(*)[128])dyn;
    __shared__ uint64_t bv[NT];
    __shared__ int32_t  bi[NT];
    __shared__ int32_t  sl[32];
    // 1-D grid of 4 row tiles x parts x chains, ordered part-major on the logical index and placed so that
    // consecutive logical indices share an XCD: the 4 * na workgroups staging one FB chunk read it through one L2
    wgclk_mark(A.wgclk, 0);
    const int li = xcd_swizzle(blockIdx.x, gridDim.x), tx = li & 3, tz = (li >> 2) % A.na, ty = (li >> 2) / A.na;
    const int nparts = gridDim.x / (4 * A.na);
    const StepChain C = A.ch[tz];
    const int t = threadIdx.x, c = C.chain;
    const int lead = tx == 0 && ty == 0;
    if (C.nb_sel < 0 && !lead) return; // finalize-only entry: one workgroup
    const int f0 = ty * A.chunk;
    uint64_t *sbest = dyn + (size_t)A.chunk * 128;
    // 0. every global load of the step issued before anything waits on one: the previous call's totals, this
    // workgroup's FB chunk (clamped into the allocated table, not the live count, so no load waits for the count)
    // and the live count and width flag.  The chunk stays in named registers (not an array: VGPRs, not scratch)
    // through the argmin and lands in LDS after it (<= PICK_CHUNK * 64 / NT each)
    uint64_t tv[4096 / NT];
    {
        const uint64_t *tot = A.tot + ((size_t)((A.step + 2) % 3) * MAX_CHAINS + c) * 4096;
#pragma unroll
        for (int u = 0; u < 4096 / NT; u++) tv[u] = C.prev_nb_sel >= 0 ? tot[u * NT + t] : 0;
    }
    static_assert(PICK_CHUNK * 64 / NT == 12, "twelve staging registers per lane");
    const uint4 *src = (const uint4 *)(A.wmse + (size_t)f0 * 128);
    const int    lim = min(A.chunk, A.fb_alloc - f0) * 64 - 1; // f0 < fb_alloc: the grid covers the table
#define LD(u) const uint4 v##u = src[min(t + (u) * NT, lim)];
    LD(0) LD(1) LD(2) LD(3) LD(4) LD(5) LD(6) LD(7) LD(8) LD(9) LD(10) LD(11)
#undef LD
    const int nfb  = C.nb_sel < 0 ? 0 : min(*A.count - f0, A.chunk);
    const int wide = *A.wide;
    wgclk_mark(A.wgclk, 1);
    // 1. selection entering this call
    if (t < 32) sl[t] = A.step ? A.lev[((size_t)(A.step - 1) * MAX_CHAINS + c) * 32 + t] : 0;
    if (C.prev_nb_sel >= 0) {
        tot_argmin(tv, A.start_gi, A.end_gi, bv, bi);
        if (t == 0) {
            const bool any = bi[0] < (1 << 30); // no candidate: (1 << 63, 0, 0) like the reference
            sl[C.prev_nb_sel]      = any ? bi[0] >> 6 : 0;
            sl[16 + C.prev_nb_sel] = any ? bi[0] & 63 : 0;
            if (C.prev_shift)
                for (int q = 0; q < C.nb - 1; q++) {
                    sl[q]      = sl[q + 1];
                    sl[16 + q] = sl[16 + q + 1];
                }
            if (lead && C.nb_sel < 0) A.best[c] = any ? bv[0] : ((uint64_t)1 << 63);
        }
    }
    if (nfb > 0) {
        uint4 *dst = (uint4 *)dyn;
#define ST(u) \
    if (t + (u) * NT < nfb * 64) dst[t + (u) * NT] = v##u;
        ST(0) ST(1) ST(2) ST(3) ST(4) ST(5) ST(6) ST(7) ST(8) ST(9) ST(10) ST(11)
#undef ST
    }
    __syncthreads();
    if (C.nb_sel < 0) { // the chain's last call has finished: publish its list
        if (t < 32) A.fin[c * 32 + t] = sl[t];
        return;
    }
    wgclk_mark(A.wgclk, 2);
    if (lead && t < 32) A.lev[((size_t)A.step * MAX_CHAINS + c) * 32 + t] = sl[t];
    // 2. zero this workgroup's slice of the accumulator used by the next step
    {
        uint64_t *nxt = A.tot + ((size_t)((A.step + 1) % 3) * MAX_CHAINS + c) * 4096;
        const int nwg = 4 * nparts, wg = ty * 4 + tx;
        for (int e = wg * NT + t; e < 4096; e += nwg * NT) nxt[e] = 0;
    }
    if (nfb <= 0) return;
    // 3. per-FB best over the selection (EbEncCdef.c:645-651)
    if (t < nfb) {
        uint64_t b = (uint64_t)1 << 63;
        for (int g = 0; g < C.nb_sel; g++) {
            const uint64_t v = m[t][sl[g]] + m[t][64 + sl[16 + g]];
            b = v < b ? v : b;
        }
        sbest[t] = b;
    }
    __syncthreads();
    wgclk_mark(A.wgclk, 3);
    // 4. accumulate.  When every entry is < 2^31 (the usual case: the check is in pick_gather_kernel), m0 + m1
    // and the min stay in 32 bits and only the running sum is 64-bit: 4 ALU ops per term instead of 7
    const int k = t & 63, j0 = 16 * tx + 4 * (t >> 6);
    uint64_t  acc[4] = {0, 0, 0, 0};
    if (!wide) {
        const uint32_t *m32 = (const uint32_t *)dyn; // low words: entry e of the chunk at m32[2 * e]
        auto term = [&](int f) {
            const uint64_t b64 = sbest[f];
            const uint32_t b = b64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)b64, m1k = m32[2 * (f * 128 + 64 + k)];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t v = m32[2 * (f * 128 + j0 + u)] + m1k;
                acc[u] += min(v, b);
            }
        };
        int f = 0;
        for (; f + 4 <= nfb; f += 4) { // 4 FBs per iteration: their LDS reads issue together
#pragma unroll
            for (int q = 0; q < 4; q++) term(f + q);
        }
        for (; f < nfb; f++) term(f);
    } else {
        for (int f = 0; f < nfb; f++) {
            const uint64_t b = sbest[f], m1k = m[f][64 + k];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t v = m[f][j0 + u] + m1k;
                acc[u] += v < b ? v : b;
            }
        }
    }
    wgclk_mark(A.wgclk, 4);
    uint64_t *cur = A.tot + ((size_t)(A.step % 3) * MAX_CHAINS + c) * 4096;
    if (k >= A.start_gi && k < A.end_gi)
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (j0 + u >= A.start_gi && j0 + u < A.end_gi)
                atomicAdd((unsigned long long *)&cur[(j0 + u) * 64 + k], (unsigned long long)acc[u]);
    if (A.wgclk) {
        __syncthreads();
        wgclk_mark(A.wgclk, 5);
    }
}

// ---- RD choice over the number of signalled strengths (EbEncCdef.c:853-872) ----
struct PickOut {
    int32_t  sb_count, nbits;
    int32_t  gi[32]; // [0, 16) luma, [16, 32) chroma strength indices of the chosen list (zero past nb)
    uint64_t best[MAX_CHAINS];
};
__global__ void pick_finish_kernel(const uint64_t *best, const int32_t *fin, const int32_t *count, uint64_t lambda,
                                   int32_t *gis, int32_t *nb_out, PickOut *out) {
    if (threadIdx.x != 0) return;
    const int sb_count  = *count;
    uint64_t  best_cost = (uint64_t)1 << 63;
    int       nbits = 0, chosen = -1; // no list chosen: the strengths stay zero
    for (int i = 0; i <= 3; i++) {
        const int      nb   = 1 << i;
        const int      bits = sb_count * i + nb * 6 * 2;
        const int64_t  rate = (int64_t)bits << 9;                                                  // av1_cost_literal
        const uint64_t cost = (uint64_t)(((rate * (int64_t)lambda + 256) >> 9) + ((int64_t)(best[i] * 16) << 7)); // RDCOST
        if (cost < best_cost) best_cost = cost, nbits = i, chosen = i;
    }
    const int nb = 1 << nbits;
    for (int j = 0; j < 16; j++) {
        gis[j]      = chosen >= 0 && j < nb ? fin[chosen * 32 + j] : 0;
        gis[16 + j] = chosen >= 0 && j < nb ? fin[chosen * 32 + 16 + j] : 0;
        out->gi[j] = gis[j], out->gi[16 + j] = gis[16 + j];
    }
    *nb_out       = nb;
    out->sb_count = sb_count;
    out->nbits    = nbits;
    for (int c = 0; c < MAX_CHAINS; c++) out->best[c] = best[c];
}

// ---- per-FB strength index (EbEncCdef.c:866-890); also into the host's copy ----
__global__ void pick_assign_kernel(const uint64_t *wmse, const int32_t *fb_list, const int32_t *count, const int32_t *d_nb,
                                   const int32_t *ygi, int8_t *fb_strength, int8_t *host_fbs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const int nb = *d_nb;
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
    if (host_fbs) host_fbs[fb_list[i]] = (int8_t)bg;
}

__global__ void fill_i8_kernel(int8_t *p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}

// FB-chunk workgroups per step across the live chains (x 4 row tiles): more parts spread the accumulation, fewer
// parts mean fewer u64 atomics into the 4096 totals (SVTGPU_PICK_PARTS for sweeps)
static int pick_parts() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_PICK_PARTS");
        return e && std::atoi(e) > 0 ? std::atoi(e) : 64;
    }();
    return v;
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
    const int sb_max = nfb; // launch shapes for every FB; the kernels read the non-skipped count on the device

    StepArgs A;
    A.wmse     = wmse;
    A.fb_alloc = nfb;
    A.count    = d_count;
    A.start_gi = 0;
    A.end_gi   = end;
    A.tot      = wmse + wmse_elems;                            // [3][4][4096]
    A.lev      = s->d_pick_lev;                                // [NSTEPS+1][4][32]
    A.fin      = s->d_pick_lev + (NSTEPS + 1) * MAX_CHAINS * 32; // [4][32]
    A.best     = s->d_pick_out;
    A.wide     = A.fin + MAX_CHAINS * 32 + 33; // after the chosen list (32) and nb
    HIP_TRY(hipMemsetAsync(A.lev, 0, sizeof(int32_t) * ((NSTEPS + 2) * MAX_CHAINS * 32 + 64), st));
    HIP_TRY(hipMemsetAsync(A.tot, 0, sizeof(uint64_t) * MAX_CHAINS * 4096, st)); // tot[0]
    hipLaunchKernelGGL(pick_gather_kernel, dim3(nfb), dim3(128), 0, st, s->d_mse, nfb, s->d_fb_list, d_count,
                       (int)ctrls->zero_fs_cost_bias, wmse, (int32_t *)A.wide);
    for (int step = 0; step <= NSTEPS; step++) {
        int na = 0;
        for (int c = 0; c < MAX_CHAINS; c++) {
            const int nb = 1 << c, len = 5 * nb; // nb calls + 4*nb refinements
            if (step > len) continue;
            StepChain &C   = A.ch[na++];
            C.chain        = c;
            C.nb           = nb;
            C.nb_sel       = step < len ? (step < nb ? step : nb - 1) : -1;
            C.prev_nb_sel  = step == 0 ? -1 : (step - 1 < nb ? step - 1 : nb - 1);
            C.prev_shift   = step >= 1 && step < len && step >= nb; // shift before calls nb.. (refinements)
        }
        A.step = step;
        // ~256 workgroups per step whatever the number of live chains (64 parts x 4 row tiles: 256 parts spent
        // more on the u64 atomics than they gained, 0.66 -> 0.59 ms per pick + apply); chunk <= PICK_CHUNK FBs
        const int want  = std::max(1, pick_parts() / std::max(na, 1));
        A.chunk         = std::min(PICK_CHUNK, std::max(4, (sb_max + want - 1) / std::max(want, 1)));
        const int parts = std::max(1, (sb_max + A.chunk - 1) / A.chunk);
        const size_t lds = (size_t)A.chunk * 129 * 8;
        A.na    = na;
        A.wgclk = svtgpu_wgclk_begin(4 * parts * na);
        hipLaunchKernelGGL(sod_step_kernel, dim3(4 * parts * na), dim3(NT), lds, st, A);
        svtgpu_wgclk_end("sod_step", 4 * parts * na, st);
    }
    HIP_TRY(hipGetLastError());
    int32_t *d_gis = A.fin + MAX_CHAINS * 32, *d_nb = d_gis + 32;
    PickOut *h_out = (PickOut *)s->h_pick;
    int8_t  *h_fbs = (int8_t *)(s->h_pick + 512);
    static_assert(sizeof(PickOut) <= 512, "pick output slot");
    hipLaunchKernelGGL(pick_finish_kernel, dim3(1), dim3(64), 0, st, (const uint64_t *)s->d_pick_out, (const int32_t *)A.fin,
                       (const int32_t *)d_count, (uint64_t)lambda, d_gis, d_nb, (PickOut *)s->h_pick_dev);
    HIP_TRY(hipMemsetAsync(s->d_fb_strength, 0, nfb, st));
    int8_t *host_fbs = fb_strength_out ? (int8_t *)(s->h_pick_dev + 512) : nullptr;
    if (host_fbs) hipLaunchKernelGGL(fill_i8_kernel, dim3((nfb + NT - 1) / NT), dim3(NT), 0, st, host_fbs, nfb);
    hipLaunchKernelGGL(pick_assign_kernel, dim3((nfb + NT - 1) / NT), dim3(NT), 0, st, wmse, s->d_fb_list, d_count, d_nb,
                       d_gis, s->d_fb_strength, host_fbs);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st)); // the only wait of the pick
    memset(params, 0, sizeof(*params));
    const int nbits = h_out->nbits, nb = 1 << nbits;
    params->cdef_bits = (uint8_t)nbits;
    for (int j = 0; j < nb; j++) {
        params->cdef_y_strength[j]  = (uint8_t)h_out->gi[j];
        params->cdef_uv_strength[j] = (uint8_t)h_out->gi[16 + j];
    }
    if (fb_strength_out) memcpy(fb_strength_out, h_fbs, nfb);
    svtgpu_count_xfer(1, sizeof(PickOut) + (fb_strength_out ? nfb : 0)); // mapped memory
    // gi -> strength code (filter_map, EbEncCdef.c:911-919); damping (:921)
    const int nf = ctrls->first_pass_fs_num;
    for (int i = 0; i < nb; i++) {
        const int y = params->cdef_y_strength[i], uv = params->cdef_uv_strength[i];
        params->cdef_y_strength[i]  = y < nf ? ctrls->default_first_pass_fs[y] : ctrls->default_second_pass_fs[y - nf];
        params->cdef_uv_strength[i] = uv < nf ? ctrls->default_first_pass_fs[uv] : ctrls->default_second_pass_fs[uv - nf];
    }
    params->cdef_damping = (uint8_t)(3 + (base_q_idx >> 6));
    return SVTGPU_OK;
}
