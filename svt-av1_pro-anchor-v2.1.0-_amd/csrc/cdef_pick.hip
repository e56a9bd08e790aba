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
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "svtgpu_internal.h"

#define NT 256
#define MAX_CHAINS 4
#define NSTEPS 40            // longest chain: nb = 8 → 8 + 32 calls (EbEncCdef.c:714-726)
#define PICK_CHUNK 48        // max FBs per workgroup (a multiple of 4; their low words staged in LDS: <= 25.7 KB)
// LDS row of a staged FB (dwords): 128 entries + 4, so the per-FB best (a lane per FB reading its row) spreads over 8
// banks instead of one, and rows stay 16-B aligned for the accumulation's quad reads
#define MROW 132

struct StepChain {
    int32_t chain;       // 0..3 (nb = 1 << chain)
    int32_t nb;
    int32_t nb_sel;      // selection size of this call (-1: finalize only)
    int32_t prev_nb_sel; // selection size of the previous call (-1: none)
    int32_t prev_shift;  // the previous call's result is followed by a refinement shift
};
struct StepArgs {
    const uint64_t *wmse;   // [sb_count][2][64] compacted, bias applied
    const uint32_t *wmse32; // the same entries' low words (what a step stages; the 64-bit path reads wmse)
    const int32_t  *count;  // sb_count, the number of non-skipped FBs (device)
    const int32_t  *wide;   // nonzero when some wmse entry is >= 2^31 (the 32-bit path would not be exact)
    int32_t         chunk, start_gi, end_gi, step, na; // na: chains in this launch
    int32_t         fb_alloc;                           // FB rows the wmse table holds
    uint64_t       *tot;    // [3][4][4096] rotating tot_mse accumulators
    int32_t        *lev;    // [NSTEPS+1][4][32] selection list entering each call
    int32_t        *fin;    // [4][32] final list per chain
    uint64_t       *best;   // [4] value returned by each chain's last call
    uint64_t       *val;    // [NSTEPS+1][4] value of the call before each step (the period shortcut's copy source)
    StepChain       ch[MAX_CHAINS];
    unsigned long long *wgclk; // diagnostics or null
    const int32_t  *skip;   // asynchronous pick, the steps after the settle check: nonzero = every chain settled, exit
};

// ---- compaction: non-skipped FBs in raster order, zero-strength bias (EbEncCdef.c:820-851) ----
__global__ void pick_compact_kernel(const uint8_t *skip, int nfb, int32_t *fb_list, int32_t *count, int32_t *wide,
                                    int32_t *fb_inv) {
    __shared__ int32_t base;
    __shared__ int32_t wsum[NT / 64];
    if (threadIdx.x == 0) base = 0, *wide = 0; // the gather raises the width flag
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
        if (fb < nfb) fb_inv[fb] = keep ? off + pre : -1; // FB -> its row in the compacted tables
        __syncthreads();
        if (threadIdx.x == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = base;
}

__global__ void pick_gather_kernel(const uint64_t *mse, int nfb, const int32_t *fb_list, const int32_t *count,
                                   int bias, uint64_t *wmse, uint32_t *wmse32, int32_t *wide, uint64_t *tot0) {
    const int i = blockIdx.x;
    if (tot0) // the first step's accumulators (launch path), spread over the grid
        for (int e = i * 128 + threadIdx.x; e < MAX_CHAINS * 4096; e += gridDim.x * 128) tot0[e] = 0;
    if (i >= *count) return;
    const int fb = fb_list[i];
    const int p = threadIdx.x >> 6, g = threadIdx.x & 63; // 128 threads
    uint64_t  v = mse[((size_t)p * nfb + fb) * 64 + g];
    if (bias && g == 0) v = ((uint64_t)bias * v) >> 6;
    wmse[((size_t)i * 2 + p) * 64 + g]   = v;
    wmse32[((size_t)i * 2 + p) * 64 + g] = (uint32_t)v;
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
    // [chunk][128] low words of the mse rows + [chunk] best (half the 64-bit rows): when other frames' kernels hold
    // most of a CU's LDS, a step's workgroups find room beside them
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn[];
    const uint32_t *m32 = (const uint32_t *)dyn; // entry e of FB f of the chunk at m32[f * MROW + e]
    __shared__ uint64_t bv[NT / 64];
    __shared__ int32_t  bi[NT / 64];
    __shared__ int32_t  sl[32];
    // 1-D grid of 4 row tiles x parts x chains, ordered part-major on the logical index and placed so that
    // consecutive logical indices share an XCD: the 4 * na workgroups staging one FB chunk read it through one L2
    if (A.skip && *A.skip) return; // uniform: the settle check wrote the final lists (svtgpu_cdef_pick_async)
    wgclk_mark(A.wgclk, 0);
    const int li = xcd_swizzle(blockIdx.x, gridDim.x), tx = li & 3, tz = (li >> 2) % A.na, ty = (li >> 2) / A.na;
    const int nparts = gridDim.x / (4 * A.na);
    const StepChain C = A.ch[tz];
    const int t = threadIdx.x, c = C.chain;
    const int lead = tx == 0 && ty == 0;
    if (C.nb_sel < 0 && !lead) return; // finalize-only entry: one workgroup
    const int f0 = ty * A.chunk;
    uint64_t *sbest = dyn + (size_t)A.chunk * (MROW / 2);
    // the period shortcut.  A chain's refinement calls (EbEncCdef.c:714-726) are a deterministic function of the
    // ordered selection entering them (entries [0, nb - 1) of lev[s]); once the selection entering call s equals the
    // one entering call s - nb, calls s, s + 1, ... repeat calls s - nb, ... result for result (the greedy loop has
    // settled into re-adding what it drops), so they are copied instead of recomputed: every workgroup reads the same
    // two lists and makes the same decision.  lp = lev[s - 1 - nb] (the previous call's period twin), lr = lev[s - nb]
    // (whose slot nb - 1 holds the twin's result).  These loads go first: a repeat is known as soon as they land, and
    // then only the chain's lead workgroup stays (to write the step's list and value; no other has work)
    const int s = A.step, nb = C.nb;
    int       lcur = 0, lp = 0, lr = 0;
    const bool chk_prev = C.prev_nb_sel >= 0 && s - 1 - nb >= nb, chk_cur = C.nb_sel >= 0 && s - nb >= nb;
    if ((t & 63) < 32) {
        if (chk_prev) {
            lcur = A.lev[((size_t)(s - 1) * MAX_CHAINS + c) * 32 + (t & 31)];
            lp   = A.lev[((size_t)(s - 1 - nb) * MAX_CHAINS + c) * 32 + (t & 31)];
        }
        if (chk_prev || chk_cur) lr = A.lev[((size_t)(s - nb) * MAX_CHAINS + c) * 32 + (t & 31)];
    }
    // 0. then every other global load of the step, issued before anything waits on one: the previous call's totals, this
    // workgroup's FB chunk (clamped into the allocated table, not the live count, so no load waits for the count)
    // and the live count and width flag.  The chunk (its low words: half the bytes of the 64-bit rows) stays in named
    // registers (not an array: VGPRs, not scratch) through the argmin and lands in LDS after it
    uint64_t tv[4096 / NT];
    {
        const uint64_t *tot = A.tot + ((size_t)((A.step + 2) % 3) * MAX_CHAINS + c) * 4096;
#pragma unroll
        for (int u = 0; u < 4096 / NT; u++) tv[u] = C.prev_nb_sel >= 0 ? tot[u * NT + t] : 0;
    }
    static_assert(PICK_CHUNK * 32 / NT == 6, "six staging registers per lane");
    const uint4 *src = (const uint4 *)(A.wmse32 + (size_t)f0 * 128);
    const int    lim = min(A.chunk, A.fb_alloc - f0) * 32 - 1; // f0 < fb_alloc: the grid covers the table
#define LD(u) const uint4 v##u = src[min(t + (u) * NT, lim)];
    LD(0) LD(1) LD(2) LD(3) LD(4) LD(5)
#undef LD
    const int  nfb  = C.nb_sel < 0 ? 0 : min(*A.count - f0, A.chunk);
    const int  wide = *A.wide;
    const bool in_state = (t & 15) < nb - 1 && (t & 63) < 32; // lanes holding entries [0, nb - 1) of both halves
    const bool prev_rep = chk_prev && !__ballot(in_state && lcur != lp);
    if (prev_rep && !lead) return; // a repeated previous call makes this one a repeat too
    wgclk_mark(A.wgclk, 1);
    // 1. selection entering this call
    if (t < 32) sl[t] = A.step ? A.lev[((size_t)(A.step - 1) * MAX_CHAINS + c) * 32 + t] : 0;
    if (C.prev_nb_sel >= 0) {
        uint64_t pv;
        int      pj, pk;
        if (prev_rep) { // the previous call repeated its twin: the twin's result and value
            pj = __shfl(lr, nb - 1), pk = __shfl(lr, 16 + nb - 1);
            pv = A.val[(size_t)(s - nb) * MAX_CHAINS + c];
        } else {
            tot_argmin(tv, A.start_gi, A.end_gi, bv, bi);
            const bool any = bi[0] < (1 << 30); // no candidate: (1 << 63, 0, 0) like the reference
            pj = any ? bi[0] >> 6 : 0, pk = any ? bi[0] & 63 : 0;
            pv = any ? bv[0] : ((uint64_t)1 << 63);
        }
        if (t == 0) {
            sl[C.prev_nb_sel]      = pj;
            sl[16 + C.prev_nb_sel] = pk;
            if (C.prev_shift)
                for (int q = 0; q < C.nb - 1; q++) {
                    sl[q]      = sl[q + 1];
                    sl[16 + q] = sl[16 + q + 1];
                }
            if (lead) A.val[(size_t)s * MAX_CHAINS + c] = pv;
            if (lead && C.nb_sel < 0) A.best[c] = pv;
        }
    }
    if (nfb > 0) {
        uint4 *dst = (uint4 *)dyn; // the low words (the 64-bit path reads the table itself), rows MROW dwords apart
#define ST(u) \
    if (t + (u) * NT < nfb * 32) dst[((t + (u) * NT) >> 5) * (MROW / 4) + ((t + (u) * NT) & 31)] = v##u;
        ST(0) ST(1) ST(2) ST(3) ST(4) ST(5)
#undef ST
    }
    __syncthreads();
    if (C.nb_sel < 0) { // the chain's last call has finished: publish its list
        if (t < 32) A.fin[c * 32 + t] = sl[t];
        return;
    }
    wgclk_mark(A.wgclk, 2);
    if (lead && t < 32) A.lev[((size_t)A.step * MAX_CHAINS + c) * 32 + t] = sl[t];
    // this call repeats its twin: nothing to accumulate (nor to zero: the chain's later calls repeat too)
    if (chk_cur && !__ballot(in_state && sl[t & 31] != lr)) return;
    // 2. zero this workgroup's slice of the accumulator used by the next step
    {
        uint64_t *nxt = A.tot + ((size_t)((A.step + 1) % 3) * MAX_CHAINS + c) * 4096;
        const int nwg = 4 * nparts, wg = ty * 4 + tx;
        for (int e = wg * NT + t; e < 4096; e += nwg * NT) nxt[e] = 0;
    }
    if (nfb <= 0) return;
    // 3. per-FB best over the selection (EbEncCdef.c:645-651)
    const uint64_t *gm = A.wmse + (size_t)f0 * 128; // the chunk's full entries (64-bit path)
    if (t < nfb) {
        uint64_t b = (uint64_t)1 << 63;
        for (int g = 0; g < C.nb_sel; g++) {
            const uint64_t v = wide ? gm[t * 128 + sl[g]] + gm[t * 128 + 64 + sl[16 + g]]
                                    : (uint64_t)m32[t * MROW + sl[g]] + m32[t * MROW + 64 + sl[16 + g]];
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
        auto term = [&](int f) {
            const uint64_t b64 = sbest[f];
            const uint32_t b = b64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)b64, m1k = m32[f * MROW + 64 + k];
            const uint4    m0 = *(const uint4 *)&m32[f * MROW + j0]; // j0 and MROW are multiples of 4
            acc[0] += min(m0.x + m1k, b), acc[1] += min(m0.y + m1k, b);
            acc[2] += min(m0.z + m1k, b), acc[3] += min(m0.w + m1k, b);
        };
        int f = 0;
        for (; f + 4 <= nfb; f += 4) { // 4 FBs per iteration: their LDS reads issue together
#pragma unroll
            for (int q = 0; q < 4; q++) term(f + q);
        }
        for (; f < nfb; f++) term(f);
    } else {
        for (int f = 0; f < nfb; f++) { // entries >= 2^31 somewhere in the frame: the full entries from the table
            const uint64_t b = sbest[f], m1k = gm[f * 128 + 64 + k];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t v = gm[f * 128 + j0 + u] + m1k;
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

// ---- the same greedy chains in one persistent launch ----
// PS_GRID workgroups stay resident for all NSTEPS + 1 steps: workgroup (chunk ci, row group g) keeps FB chunk ci
// (<= PS_CH FBs) in LDS from the first step to the last and accumulates rows 16 g .. 16 g + 15 of every live chain's
// tot over it.  A step is two exchanges through tagged 64-bit words (an 8-bit tag of the pick and step above a
// 56-bit value, stored and polled with agent-scope atomics: a word is valid by itself, no fence or counter):
//   1. the partial sums of every chunk -> the workgroup that owns row j of chain c sums its 64 entries over the 64
//      chunks and publishes the row's first minimum (value, index);
//   2. every workgroup reads the rows' minima of every live chain and takes the first minimum of the call
//      (svt_search_one_dual's final loop, EbEncCdef.c:670-679), which every workgroup folds into the same selection.
// The words of one exchange are rewritten at every step before anyone can read the next step's (a workgroup
// reaches step s + 1 only after every row owner has read step s), so one buffer serves all steps; the pick's
// 2-bit epoch in the tag keeps the previous pick's words apart.  Co-residency: PS_GRID workgroups of <= 34 KB
// LDS and 256 threads (several fit per CU, and a pick launched beside another finds room); a poll gives up after
// a bounded wait and sets a status bit, so a grid that cannot drain still ends.  Partial sums fit 56 bits:
// an entry is < 2^41 (a 64x64 block's SSE at 12 bits is < 2^37), a chunk sums <= PS_CH of them, a total <= 2^15.
#define PS_GRID  256
#define PS_NCH   64  // FB chunks (x 4 row groups = PS_GRID)
#define PS_CH    32  // FBs per chunk at most: frames up to 2048 non-skipped 64x64 blocks (3840x2160: 2040)
constexpr unsigned long long PS_LOW = (1ull << 56) - 1;

struct PersistArgs {
    const uint64_t     *wmse;   // [fb_alloc][2][64] compacted, bias applied
    const int32_t      *count;  // live FB count (device)
    const int32_t      *wide;   // some entry >= 2^31: 64-bit terms
    int32_t             chunk, fb_alloc, end_gi;
    uint32_t            epoch;  // low 2 bits tag this pick's words
    unsigned long long *part;   // [PS_NCH][4][4096] tagged partial sums
    unsigned long long *amin;   // [4][64][2] tagged row minima: value, index
    int32_t            *fin;    // [4][32] final list per chain
    uint64_t           *best;   // [4]
    int32_t            *status; // bit 0: a poll gave up
    unsigned long long *stat;   // diagnostics (SVTGPU_PICK_STATS) or null: ticks of compute, exchange 1, exchange 2
    const int32_t      *skip;   // the asynchronous pick's fallback: nonzero = every chain settled at the check, exit
    const uint32_t     *dep;    // ... its epoch, counted on the device (the check raises it when this launch will run)
};

// chain c's call at step s (the host schedule of the launch path): nb_sel = selection size of this call (-1: the
// chain finished with the previous call; -2: the chain ended before), prev = the previous call's size (-1: none)
struct ChainStep {
    int nb, nb_sel, prev, shift;
};
__device__ __forceinline__ ChainStep chain_step(int c, int step) {
    const int nb = 1 << c, len = 5 * nb;
    ChainStep r;
    r.nb     = nb;
    r.nb_sel = step > len ? -2 : step < len ? (step < nb ? step : nb - 1) : -1;
    r.prev   = step == 0 || step > len ? -1 : (step - 1 < nb ? step - 1 : nb - 1);
    r.shift  = step >= 1 && step < len && step >= nb;
    return r;
}

// poll the N tagged words p[i * stride] (those with use set) until every tag matches; false after the bounded wait
template <int N>
__device__ __forceinline__ bool ps_poll(const unsigned long long *p, size_t stride, bool use, unsigned long long (&v)[N],
                                        unsigned long long tag) {
    if (!use) return true;
    uint32_t pend = (1u << N) - 1; // words still to see: a re-poll loads only those
    for (unsigned spin = 0;; spin++) {
#pragma unroll
        for (int i = 0; i < N; i++)
            if (pend >> i & 1) {
                v[i] = __hip_atomic_load(p + i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((v[i] & ~PS_LOW) == tag) pend &= ~(1u << i);
            }
        if (!pend) return true;
        if (spin > (1u << 20)) return false; // ~0.1 s
        __builtin_amdgcn_s_sleep(4);
    }
}

// the sum of the N tagged words p[i * stride] (their 56-bit values), each added once its tag is seen
template <int N>
__device__ __forceinline__ bool ps_poll_sum(const unsigned long long *p, size_t stride, unsigned long long tag,
                                            unsigned long long &sum) {
    uint32_t pend = (1u << N) - 1;
    sum           = 0;
    for (unsigned spin = 0;; spin++) {
#pragma unroll
        for (int i = 0; i < N; i++)
            if (pend >> i & 1) {
                const unsigned long long v = __hip_atomic_load(p + i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((v & ~PS_LOW) == tag) pend &= ~(1u << i), sum += v & PS_LOW;
            }
        if (!pend) return true;
        if (spin > (1u << 20)) return false; // ~0.1 s
        __builtin_amdgcn_s_sleep(4);
    }
}

__device__ __forceinline__ void ps_store(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(NT, 4) sod_persist_kernel(const PersistArgs A) {
    __shared__ __attribute__((aligned(16))) uint64_t m64[PS_CH * 128]; // the chunk: u64 rows, or u32 rows (narrow)
    __shared__ uint64_t sb[MAX_CHAINS][PS_CH];                          // per-FB best over each chain's selection
    __shared__ int32_t  sl[MAX_CHAINS][32];                             // selections ([0,16) luma, [16,32) chroma)
    __shared__ uint64_t red[NT];
    __shared__ int      s_fail;
    const uint32_t *m32 = (const uint32_t *)m64;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int li = xcd_swizzle(blockIdx.x, gridDim.x), ci = li >> 2, g = li & 3; // a chunk's 4 groups share an XCD
    const int f0 = ci * A.chunk, end = A.end_gi;
    const int nfb  = max(0, min(*A.count - f0, A.chunk));
    const int wide = *A.wide;
    if (A.skip && *A.skip) return; // uniform: the settle check finished the pick (svtgpu_cdef_pick_async)
    const unsigned long long ep = (unsigned long long)((A.dep ? *A.dep : A.epoch) & 3) << 62;
    unsigned long long       tk[3] = {0, 0, 0}, t0 = 0;
    if (t == 0) s_fail = 0;
    // the chunk into LDS, once (narrow: the low words, entry e of FB f at m32[f * 128 + e])
    for (int e = t; e < nfb * 128; e += NT) {
        const uint64_t v = A.wmse[(size_t)f0 * 128 + e];
        if (wide) m64[e] = v;
        else ((uint32_t *)m64)[e] = (uint32_t)v;
    }
    if (t < MAX_CHAINS * 32) sl[t >> 5][t & 31] = 0;
    __syncthreads();
    for (int step = 0; step <= NSTEPS; step++) {
        const unsigned long long tag = ep | (unsigned long long)(step + 1) << 56, ptag = ep | (unsigned long long)step << 56;
        if (A.stat && t == 0) t0 = __builtin_amdgcn_s_memrealtime();
        // 1. the previous call's first minimum per chain (wave c: lane j holds row j's minimum), folded into the
        // selection; a finishing chain publishes its list and value
        {
            const int       c = w;
            const ChainStep C = chain_step(c, step);
            if (C.prev >= 0) {
                unsigned long long v[2] = {PS_LOW, PS_LOW};
                if (!ps_poll<2>(A.amin + (c * 64 + lane) * 2, 1, lane < end, v, ptag)) s_fail = 1;
                unsigned long long bv = v[0] & PS_LOW;
                int                bi = (v[1] & PS_LOW) == PS_LOW ? (1 << 30) : (int)(v[1] & PS_LOW);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long ov = __shfl_xor(bv, o);
                    const int                oi = __shfl_xor(bi, o);
                    if (ov < bv || (ov == bv && oi < bi)) bv = ov, bi = oi;
                }
                if (lane == 0) {
                    const bool any = bi < (1 << 30);
                    sl[c][C.prev]      = any ? bi >> 6 : 0;
                    sl[c][16 + C.prev] = any ? bi & 63 : 0;
                    if (C.shift)
                        for (int q = 0; q < C.nb - 1; q++) sl[c][q] = sl[c][q + 1], sl[c][16 + q] = sl[c][16 + q + 1];
                    if (li == 0 && C.nb_sel == -1) A.best[c] = any ? bv : ((uint64_t)1 << 63);
                }
            }
        }
        __syncthreads();
        if (li == 0 && t < MAX_CHAINS * 32 && chain_step(t >> 5, step).nb_sel == -1) A.fin[t] = sl[t >> 5][t & 31];
        if (step == NSTEPS) break; // the last step only finishes the longest chain
        if (A.stat && t == 0) tk[2] += __builtin_amdgcn_s_memrealtime() - t0, t0 = __builtin_amdgcn_s_memrealtime();
        // 2. per-FB best over each live chain's selection (EbEncCdef.c:645-651): wave c, lane f
        {
            const int       c = w;
            const ChainStep C = chain_step(c, step);
            if (C.nb_sel >= 0 && lane < nfb) {
                uint64_t b = (uint64_t)1 << 63;
                for (int q = 0; q < C.nb_sel; q++) {
                    const int      j = sl[c][q], k = sl[c][16 + q];
                    const uint64_t v = wide ? m64[lane * 128 + j] + m64[lane * 128 + 64 + k]
                                            : (uint64_t)m32[lane * 128 + j] + m32[lane * 128 + 64 + k];
                    b = v < b ? v : b;
                }
                sb[c][lane] = b;
            }
        }
        __syncthreads();
        // 3. partial sums of rows 16 g + 4 w + {0..3}, column k = lane, of every live chain over the chunk
        const int j0 = 16 * g + 4 * w, k = lane;
#pragma unroll 1
        for (int c = 0; c < MAX_CHAINS; c++) {
            if (chain_step(c, step).nb_sel < 0) continue;
            uint64_t acc[4] = {0, 0, 0, 0};
            if (!wide) {
#pragma unroll 4
                for (int f = 0; f < nfb; f++) {
                    const uint64_t b64 = sb[c][f];
                    const uint32_t b = b64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)b64, m1k = m32[f * 128 + 64 + k];
                    const uint4    m0 = *(const uint4 *)&m32[f * 128 + j0];
                    acc[0] += min(m0.x + m1k, b), acc[1] += min(m0.y + m1k, b);
                    acc[2] += min(m0.z + m1k, b), acc[3] += min(m0.w + m1k, b);
                }
            } else {
#pragma unroll 1
                for (int f = 0; f < nfb; f++) {
                    const uint64_t b = sb[c][f], m1k = m64[f * 128 + 64 + k];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint64_t v = m64[f * 128 + j0 + u] + m1k;
                        acc[u] += v < b ? v : b;
                    }
                }
            }
            if (k < end)
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (j0 + u < end) ps_store(A.part + ((size_t)(ci * 4 + c) * 4096 + (j0 + u) * 64 + k), tag | acc[u]);
        }
        if (A.stat && t == 0) tk[0] += __builtin_amdgcn_s_memrealtime() - t0, t0 = __builtin_amdgcn_s_memrealtime();
        // 4. row owners: row j of the a-th live chain belongs to workgroup a * 64 + j (a < live chains, j < end)
        {
            int na = 0, c = -1;
            for (int q = 0; q < MAX_CHAINS; q++)
                if (chain_step(q, step).nb_sel >= 0) {
                    if (na == (li >> 6)) c = q;
                    na++;
                }
            const int j = li & 63;
            if (c >= 0 && j < end) {
                unsigned long long s = 0;
                if (k < end && !ps_poll_sum<PS_NCH / 4>(A.part + (size_t)(w * 4 + c) * 4096 + j * 64 + k, (size_t)16 * 4096, tag, s))
                    s_fail = 1;
                red[t] = s;
                __syncthreads();
                if (w == 0) {
                    unsigned long long bv = PS_LOW;
                    int                bi = 1 << 30;
                    if (k < end) bv = red[k] + red[64 + k] + red[128 + k] + red[192 + k], bi = j * 64 + k;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        const unsigned long long ov = __shfl_xor(bv, o);
                        const int                oi = __shfl_xor(bi, o);
                        if (ov < bv || (ov == bv && oi < bi)) bv = ov, bi = oi;
                    }
                    if (lane == 0) {
                        ps_store(A.amin + (c * 64 + j) * 2, tag | (bv & PS_LOW));
                        ps_store(A.amin + (c * 64 + j) * 2 + 1, tag | (unsigned long long)bi);
                    }
                }
            }
        }
        if (A.stat && t == 0) tk[1] += __builtin_amdgcn_s_memrealtime() - t0;
    }
    __syncthreads();
    if (t == 0 && s_fail) atomicOr(A.status, 1);
    if (A.stat && t == 0 && li == 0) A.stat[0] += tk[0], A.stat[1] += tk[1], A.stat[2] += tk[2], A.stat[3] += 1;
}

// ---- the settle check: the launch path's steps after T skipped when every chain has settled by then ----
// After step T's launch every chain c (nb = 1 << c, calls 0 .. L - 1, L = 5 nb) has either finished (L <= T) or
// entered call T with the selection lev[T].  If lev[T]'s state (entries [0, nb - 1) of both halves) equals lev[T - nb]'s
// with T - nb >= nb, the chain repeats with period nb from call T - nb on (sod_step_kernel's period shortcut), so its
// last call L - 1 equals call a = T - nb + (L - 1 - T + nb) mod nb: the final list is lev[a] with slot nb - 1 taken from
// lev[b] (b = the period twin of L: lev[t][nb - 1] is the result of call t - 1) and the value val[a + 1] -- exactly what
// steps T + 1 .. L would produce.  One lane per chain; out[0] = 1 when every unfinished chain settled (their fin / best
// written), out[1] = the latest step at which a chain that needs one settled (or finished): the host's next T.
struct SettleOut {
    int32_t settled, step, seq; // seq: the asynchronous pick that wrote it (its next T is read without a wait)
};
// flag (device memory, asynchronous pick): the settled word the later steps read
// dep: the persistent fallback's epoch (asynchronous pick), raised when the check finds a chain unsettled -- only then
// does the fallback launch run, so its exchange words' epochs differ from those of its last four real runs
__global__ void pick_settle_kernel(const int32_t *lev, const uint64_t *val, int32_t *fin, uint64_t *best, int T,
                                   SettleOut *out, int32_t *flag, int seq, uint32_t *dep) {
    __shared__ int s_ok[MAX_CHAINS], s_at[MAX_CHAINS];
    const int c = threadIdx.x;
    if (c < MAX_CHAINS) {
        const int nb = 1 << c, L = 5 * nb;
        auto lv   = [&](int s, int i) { return lev[((size_t)s * MAX_CHAINS + c) * 32 + i]; };
        auto same = [&](int s1, int s2) {
            for (int q = 0; q < nb - 1; q++)
                if (lv(s1, q) != lv(s2, q) || lv(s1, 16 + q) != lv(s2, 16 + q)) return false;
            return true;
        };
        int at = L; // the first step from which the chain repeats (L: it finishes first)
        for (int st = 2 * nb; st <= min(T, L - 1); st++)
            if (same(st, st - nb)) {
                at = st;
                break;
            }
        bool ok = L <= T || at <= T;
        if (L > T && ok) {
            const int base = T - nb, a = base + (L - 1 - base) % nb, b = base + (L - base) % nb;
            for (int i = 0; i < 32; i++) fin[c * 32 + i] = lv(a, i);
            fin[c * 32 + nb - 1]      = lv(b, nb - 1);
            fin[c * 32 + 16 + nb - 1] = lv(b, 16 + nb - 1);
            best[c]                   = val[(size_t)(a + 1) * MAX_CHAINS + c];
        }
        s_ok[c] = ok, s_at[c] = at;
    }
    __syncthreads();
    if (c == 0) {
        const int ok = s_ok[0] && s_ok[1] && s_ok[2] && s_ok[3];
        if (flag) *flag = ok;
        if (dep && !ok) *dep += 1;
        out->settled = ok;
        out->step    = max(max(s_at[0], s_at[1]), max(s_at[2], s_at[3]));
        if (seq) {
            __threadfence_system();
            __hip_atomic_store(&out->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---- RD choice over the number of signalled strengths (EbEncCdef.c:853-872) ----
struct PickOut {
    int32_t  sb_count, nbits, status, seq; // seq: the asynchronous pick that wrote it (0: a synchronous one)
    int32_t  gi[32]; // [0, 16) luma, [16, 32) chroma strength indices of the chosen list (zero past nb)
    uint64_t best[MAX_CHAINS];
};
// the asynchronous pick's conversion of the chosen list into the frame parameters: strength index gi -> its code
// (filter_map, EbEncCdef.c:911-919), the damping (:921)
struct PickMap {
    uint8_t code[64];
    uint8_t damping;
};
__global__ void pick_final_kernel(const uint64_t *best, const int32_t *fin, const int32_t *count, uint64_t lambda,
                                  PickOut *out, int32_t *status, const uint64_t *wmse, const int32_t *fb_inv, int nfb,
                                  int8_t *fb_strength, int8_t *host_fbs, SvtGpuCdefParams *dprm, const PickMap map,
                                  int seq) {
    __shared__ int32_t gi[32];
    __shared__ int32_t s_nb;
    const int t = threadIdx.x;
    if (t == 0) { // every workgroup makes the same choice; workgroup 0 publishes it
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
            gi[j]      = chosen >= 0 && j < nb ? fin[chosen * 32 + j] : 0;
            gi[16 + j] = chosen >= 0 && j < nb ? fin[chosen * 32 + 16 + j] : 0;
        }
        s_nb = nb;
        if (blockIdx.x == 0) {
            for (int j = 0; j < 32; j++) out->gi[j] = gi[j];
            out->sb_count = sb_count;
            out->nbits    = nbits;
            for (int c = 0; c < MAX_CHAINS; c++) out->best[c] = best[c];
            out->status = *status; // the persistent kernel's (0 on the launch path), re-armed for the next pick
            *status     = 0;
            if (dprm) { // the parameters the apply reads (svtgpu_cdef_apply_frame with params == NULL)
                SvtGpuCdefParams q;
                memset(&q, 0, sizeof q);
                q.cdef_damping = map.damping, q.cdef_bits = (uint8_t)nbits;
                for (int j = 0; j < nb; j++) q.cdef_y_strength[j] = map.code[gi[j]], q.cdef_uv_strength[j] = map.code[gi[16 + j]];
                *dprm = q;
            }
            if (seq) {
                __threadfence_system();
                __hip_atomic_store(&out->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    __syncthreads();
    // per-FB strength index (EbEncCdef.c:866-890), skipped FBs 0; also into the host's copy
    const int fb = blockIdx.x * blockDim.x + t;
    if (fb >= nfb) return;
    const int i  = fb_inv[fb];
    int       bg = 0;
    if (i >= 0) {
        const uint64_t *m0 = wmse + (size_t)i * 128, *m1 = m0 + 64;
        uint64_t        bc = (uint64_t)1 << 63;
        for (int g = 0; g < s_nb; g++) {
            const uint64_t c = m0[gi[g]] + m1[gi[16 + g]];
            if (c < bc) bc = c, bg = g;
        }
    }
    fb_strength[fb] = (int8_t)bg;
    if (host_fbs) host_fbs[fb] = (int8_t)bg;
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

// FBs per workgroup at most (SVTGPU_PICK_CHUNK, a multiple of 4 up to PICK_CHUNK, for sweeps)
static int pick_chunk() {
    static const int v = [] {
        const char *e = std::getenv("SVTGPU_PICK_CHUNK");
        const int   c = e ? std::atoi(e) : 0;
        return c >= 4 && c <= PICK_CHUNK ? c & ~3 : PICK_CHUNK;
    }();
    return v;
}

void cdef_pick_host_result(SvtGpuCdefFrameState *s, const PickMap &map, SvtGpuCdefParams *params,
                           int8_t *fb_strength_out);

// params == nullptr: the asynchronous pick (svtgpu_cdef_pick_async) -- no host wait: the settle check's outcome reaches
// the later steps through a device flag (they exit at once when every chain has settled), the final kernel writes the
// frame parameters to device memory for the apply, and the host reads the result later (svtgpu_cdef_read_params)
int svtgpu_cdef_pick_impl(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                          uint64_t lambda, SvtGpuCdefParams *params, int8_t *fb_strength_out, hipStream_t st) {
    const bool async_ = params == nullptr;
    const int nfb = s->nfb;
    const int end = ctrls->first_pass_fs_num + ctrls->default_second_pass_fs_num;
    if (end <= 0 || end > 64)
        return SVTGPU_ERR_INVALID_ARG;
    uint64_t *wmse = s->d_pick_part; // layout: [nfb*128] wmse, then partials
    const size_t wmse_elems = (size_t)nfb * 128;
    int32_t  *d_count = s->d_fb_list + nfb;
    StepArgs  A;
    A.lev  = s->d_pick_lev;                                  // [NSTEPS+1][4][32]
    A.fin  = s->d_pick_lev + (NSTEPS + 1) * MAX_CHAINS * 32; // [4][32]
    A.wide = A.fin + MAX_CHAINS * 32 + 33;                   // after the chosen list (32) and nb
    // the persistent launch (SVTGPU_PICK_PERSIST=1; default: the launch per step) while its chunks hold every FB
    const char *pe      = std::getenv("SVTGPU_PICK_PERSIST");
    const bool  persist = pe && pe[0] == '1' && nfb <= PS_NCH * PS_CH;
    int32_t    *d_inv   = s->d_fb_list + nfb + 1;
    A.tot               = wmse + wmse_elems;                          // [3][4][4096]
    A.val               = A.tot + (size_t)3 * MAX_CHAINS * 4096;      // [NSTEPS+1][4]
    uint32_t *wmse32    = (uint32_t *)(A.val + (NSTEPS + 1) * MAX_CHAINS); // [nfb][128] low words
    A.wmse32            = wmse32;
    hipLaunchKernelGGL(pick_compact_kernel, dim3(1), dim3(NT), 0, st, s->d_skip, nfb, s->d_fb_list, d_count,
                       (int32_t *)A.wide, d_inv);
    const int sb_max = nfb; // launch shapes for every FB; the kernels read the non-skipped count on the device

    A.wmse     = wmse;
    A.fb_alloc = nfb;
    A.count    = d_count;
    A.start_gi = 0;
    A.end_gi   = end;
    A.best     = s->d_pick_out;
    A.skip     = nullptr;
    hipLaunchKernelGGL(pick_gather_kernel, dim3(nfb), dim3(128), 0, st, s->d_mse, nfb, s->d_fb_list, d_count,
                       (int)ctrls->zero_fs_cost_bias, wmse, wmse32, (int32_t *)A.wide, persist ? nullptr : A.tot);
    unsigned long long *xch = (unsigned long long *)s->d_pick_xch, *stat = nullptr;
    int32_t            *d_status = (int32_t *)(xch + PS_NCH * 4 * 4096 + 4 * 64 * 2);
    if (persist) {
        static const bool stats = std::getenv("SVTGPU_PICK_STATS") != nullptr;
        if (s->pick_xch_end != end) { // words of a different strength count could carry a current tag
            HIP_TRY(hipMemsetAsync(xch, 0, SVTGPU_PICK_XCH_BYTES, st));
            s->pick_xch_end = end;
        }
        if (stats) stat = xch + PS_NCH * 4 * 4096 + 4 * 64 * 2 + 8;
        PersistArgs P;
        P.wmse     = wmse;
        P.count    = d_count;
        P.wide     = A.wide;
        P.chunk    = std::max(1, (nfb + PS_NCH - 1) / PS_NCH);
        P.fb_alloc = nfb;
        P.end_gi   = end;
        P.epoch    = s->pick_epoch++;
        P.part     = xch;
        P.amin     = xch + PS_NCH * 4 * 4096;
        P.fin      = A.fin;
        P.best     = A.best;
        P.status   = d_status;
        P.stat     = stat;
        P.skip     = nullptr;
        P.dep      = nullptr;
        hipLaunchKernelGGL(sod_persist_kernel, dim3(PS_GRID), dim3(NT), 0, st, P);
    }
    // the settle checkpoint (SVTGPU_PICK_SETTLE=0: off): after step T one small kernel checks whether every chain has
    // settled into its period and, if so, writes the final lists, and the host skips the remaining launches (one
    // wait instead of up to 40 - T dependent launches, each of which waits for free CU slots when other frames' kernels
    // hold the device).  T follows the last pick's settling step; an unsettled check moves it 4 steps later
    static const bool settle_on = [] {
        const char *e = std::getenv("SVTGPU_PICK_SETTLE");
        return !(e && e[0] == '0');
    }();
    SettleOut *h_settle = (SettleOut *)(s->h_pick + 448), *d_settle = (SettleOut *)(s->h_pick_dev + 448);
    static_assert(sizeof(PickOut) <= 448, "pick output slot below the settle record");
    int32_t *d_flag = (int32_t *)s->d_apick; // asynchronous: the settled word (device memory)
    if (async_) {
        // the last asynchronous check whose record has landed (read without a wait: the host may run ahead of the
        // device) moves T as the synchronous path does right after its check
        const volatile SettleOut *hs = (const volatile SettleOut *)h_settle;
        if (hs->seq != 0 && hs->seq != s->settle_seen) {
            s->settle_seen = hs->seq;
            if (hs->settled) {
                s->pick_settle = hs->step, s->pick_miss = 0;
            } else {
                s->pick_settle = std::min(s->pick_settle + 4, NSTEPS - 4);
                if (++s->pick_miss >= 2) s->pick_skip = 8, s->pick_miss = 0;
            }
        }
    }
    // after two consecutive checks that found a chain unsettled the next 8 picks skip the check (its host wait saves
    // nothing on a sequence that does not settle), then it is tried again from step 24
    const bool check = settle_on && s->pick_skip == 0;
    if (s->pick_skip > 0 && --s->pick_skip == 0) s->pick_settle = 24;
    const int T = check ? std::min(std::max(s->pick_settle, 16), NSTEPS) : NSTEPS;
    // asynchronous: after the check no further step is launched -- when a chain has not settled, one persistent launch
    // (sod_persist_kernel, which returns at once when the check's flag says settled) recomputes the whole pick.  The
    // flag-only step launches it replaces each needed 256 workgroup slots, which at four frames in flight waited for
    // CUs held by other frames' kernels.  Frames with more FBs than its chunks hold keep the flagged launches.
    const char *afb         = std::getenv("SVTGPU_PICK_ASYNC_FALLBACK"); // =steps: the flagged step launches (A/B)
    const bool  async_steps = afb && !std::strcmp(afb, "steps");
    const bool pfb = async_ && !persist && !async_steps && T < NSTEPS && nfb <= PS_NCH * PS_CH;
    if (pfb && s->pick_xch_end != end) { // words of a different strength count could carry a current tag
        HIP_TRY(hipMemsetAsync(s->d_pick_xch, 0, SVTGPU_PICK_XCH_BYTES, st));
        s->pick_xch_end = end;
    }
    for (int step = 0; step <= NSTEPS && !persist && !(pfb && step > T); step++) {
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
        A.skip = async_ && step > T ? d_flag : nullptr;
        // ~256 workgroups per step whatever the number of live chains (64 parts x 4 row tiles: 256 parts spent
        // more on the u64 atomics than they gained, 0.66 -> 0.59 ms per pick + apply); chunk <= PICK_CHUNK FBs
        const int want  = std::max(1, pick_parts() / std::max(na, 1));
        A.chunk         = std::min(pick_chunk(), std::max(4, (sb_max + want - 1) / std::max(want, 1)));
        const int parts = std::max(1, (sb_max + A.chunk - 1) / A.chunk);
        const size_t lds = (size_t)A.chunk * (MROW * 4 + 8);
        A.na    = na;
        A.wgclk = svtgpu_wgclk_begin(4 * parts * na);
        hipLaunchKernelGGL(sod_step_kernel, dim3(4 * parts * na), dim3(NT), lds, st, A);
        svtgpu_wgclk_end("sod_step", 4 * parts * na, st);
        if (step == T && T < NSTEPS && async_) { // the check in stream order; the later steps read its flag
            hipLaunchKernelGGL(pick_settle_kernel, dim3(1), dim3(64), 0, st, (const int32_t *)A.lev,
                               (const uint64_t *)A.val, A.fin, A.best, T, d_settle, d_flag, ++s->settle_seq,
                               pfb ? (uint32_t *)((uint8_t *)s->d_apick + 8) : (uint32_t *)nullptr);
            HIP_TRY(hipGetLastError());
        } else if (step == T && T < NSTEPS) {
            hipLaunchKernelGGL(pick_settle_kernel, dim3(1), dim3(64), 0, st, (const int32_t *)A.lev,
                               (const uint64_t *)A.val, A.fin, A.best, T, d_settle, (int32_t *)nullptr, 0,
                               (uint32_t *)nullptr);
            HIP_TRY(hipGetLastError());
            if (int rc = svtgpu_comm_wait(s->comm, st)) return rc; // bounded behind the tables' exchange
            svtgpu_count_xfer(1, sizeof(SettleOut));
            if (h_settle->settled) {
                s->pick_settle = h_settle->step;
                s->pick_miss   = 0;
                break;
            }
            s->pick_settle = std::min(T + 4, NSTEPS - 4); // keep checking: a later frame may settle
            if (++s->pick_miss >= 2) s->pick_skip = 8, s->pick_miss = 0;
        }
    }
    HIP_TRY(hipGetLastError());
    if (pfb) { // the fallback: the whole pick again, only when the check found a chain unsettled
        PersistArgs P;
        P.wmse     = wmse;
        P.count    = d_count;
        P.wide     = A.wide;
        P.chunk    = std::max(1, (nfb + PS_NCH - 1) / PS_NCH);
        P.fb_alloc = nfb;
        P.end_gi   = end;
        P.epoch    = 0;
        P.part     = (unsigned long long *)s->d_pick_xch;
        P.amin     = P.part + PS_NCH * 4 * 4096;
        P.fin      = A.fin;
        P.best     = A.best;
        P.status   = d_status;
        P.stat     = nullptr;
        P.skip     = d_flag;
        P.dep      = (const uint32_t *)((const uint8_t *)s->d_apick + 8);
        hipLaunchKernelGGL(sod_persist_kernel, dim3(PS_GRID), dim3(NT), 0, st, P);
        HIP_TRY(hipGetLastError());
    }
    PickOut *h_out = (PickOut *)s->h_pick;
    static_assert(sizeof(PickOut) <= 512, "pick output slot");
    int8_t *host_fbs = fb_strength_out || async_ ? (int8_t *)(s->h_pick_dev + 512) : nullptr;
    PickMap map;
    std::memset(&map, 0, sizeof map);
    const int nf = ctrls->first_pass_fs_num;
    for (int g = 0; g < end; g++) // gi -> strength code (filter_map, EbEncCdef.c:911-919)
        map.code[g] = g < nf ? ctrls->default_first_pass_fs[g] : ctrls->default_second_pass_fs[g - nf];
    map.damping = (uint8_t)(3 + (base_q_idx >> 6)); // :921
    const int seq = async_ ? ++s->apick_seq : 0;
    hipLaunchKernelGGL(pick_final_kernel, dim3((nfb + NT - 1) / NT), dim3(NT), 0, st, (const uint64_t *)s->d_pick_out,
                       (const int32_t *)A.fin, (const int32_t *)d_count, (uint64_t)lambda, (PickOut *)s->h_pick_dev,
                       d_status, (const uint64_t *)wmse, (const int32_t *)d_inv, nfb, s->d_fb_strength, host_fbs,
                       async_ ? (SvtGpuCdefParams *)((uint8_t *)s->d_apick + 16) : (SvtGpuCdefParams *)nullptr, map, seq);
    HIP_TRY(hipGetLastError());
    if (async_) {
        std::memcpy(s->apick_map, map.code, 64);
        s->apick_damping = map.damping;
        return SVTGPU_OK;
    }
    if (int rc = svtgpu_comm_wait(s->comm, st)) return rc; // the only wait of the pick (bounded when tiled)
    if (h_out->status) {
        svtgpu_set_last_hip_error(hipErrorUnknown, "CDEF pick: the persistent step exchange timed out", __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    if (stat) {
        unsigned long long v[4];
        HIP_TRY(hipMemcpy(v, stat, sizeof v, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(stat, 0, sizeof v));
        std::fprintf(stderr, "sod_persist (workgroup 0): compute+store %.1f us, reduce %.1f us, minima %.1f us\n",
                     v[0] * 0.01, v[1] * 0.01, v[2] * 0.01);
    }
    cdef_pick_host_result(s, map, params, fb_strength_out);
    return SVTGPU_OK;
}

// the pick's result from the mapped record (after the stream wait): the parameters through the strength map, the
// per-FB strengths
void cdef_pick_host_result(SvtGpuCdefFrameState *s, const PickMap &map, SvtGpuCdefParams *params,
                           int8_t *fb_strength_out) {
    const PickOut *h_out = (const PickOut *)s->h_pick;
    memset(params, 0, sizeof(*params));
    const int nbits = h_out->nbits, nb = 1 << nbits;
    params->cdef_bits    = (uint8_t)nbits;
    params->cdef_damping = map.damping;
    for (int j = 0; j < nb; j++) {
        params->cdef_y_strength[j]  = map.code[h_out->gi[j]];
        params->cdef_uv_strength[j] = map.code[h_out->gi[16 + j]];
    }
    if (fb_strength_out) memcpy(fb_strength_out, s->h_pick + 512, s->nfb);
    svtgpu_count_xfer(1, sizeof(PickOut) + (fb_strength_out ? s->nfb : 0)); // mapped memory
}

// svtgpu_cdef_read_params: the last asynchronous pick's result, after a (bounded) wait for the stream
int svtgpu_cdef_pick_read(SvtGpuCdefFrameState *s, SvtGpuCdefParams *params, int8_t *fb_strength_out, hipStream_t st) {
    if (int rc = svtgpu_comm_wait(s->comm, st)) return rc;
    s->apick_pending = 0;
    if (s->apick_ref) { // the reference-fs parameters (no search): known when the pick was enqueued
        *params = s->apick_params;
        if (fb_strength_out) memset(fb_strength_out, 0, s->nfb);
        return SVTGPU_OK;
    }
    const volatile PickOut *h_out = (const volatile PickOut *)s->h_pick;
    if (h_out->seq != s->apick_seq) {
        svtgpu_set_last_hip_error(hipErrorUnknown, "CDEF asynchronous pick: result record missing after the stream wait",
                                  __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    if (h_out->status) {
        svtgpu_set_last_hip_error(hipErrorUnknown, "CDEF pick: the persistent step exchange timed out", __FILE__, __LINE__);
        return SVTGPU_ERR_HIP;
    }
    PickMap map;
    std::memcpy(map.code, s->apick_map, 64);
    map.damping = s->apick_damping;
    cdef_pick_host_result(s, map, params, fb_strength_out);
    return SVTGPU_OK;
}
