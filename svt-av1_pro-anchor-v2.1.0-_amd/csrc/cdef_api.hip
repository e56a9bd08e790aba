// cdef_api.hip — frame-level CDEF entry points of the C ABI (include/svtgpu.h).
#include <cstdlib>
#include <algorithm>
#include <cstring>

#include "svtgpu_internal.h"

int svtgpu_cdef_pick_read(SvtGpuCdefFrameState *s, SvtGpuCdefParams *params, int8_t *fb_strength_out, hipStream_t st);
int svtgpu_cdef_pick_impl(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                          uint64_t lambda, SvtGpuCdefParams *params, int8_t *fb_strength_out, hipStream_t st);

// set_cdef_controls (Source/Lib/Encoder/Codec/EncModeConfig.c:860-1330), searched levels only.
extern "C" int svtgpu_cdef_controls_for_level(int level, SvtGpuCdefControls *c) {
    if (!c)
        return SVTGPU_ERR_INVALID_ARG;
    static const uint8_t pf_gi[16] = {0, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48, 52, 56, 60}; // :12
    struct Level {
        int         nfirst;
        uint8_t     first[16]; // indices into pf_gi
        int         nsec;      // secondary strengths per primary
        uint8_t     sec[3];    // secondary codes added to the primary code
        bool        sec_uv;    // second-pass chroma tested
        uint8_t     ss;
        uint16_t    bias;
    };
    Level L{};
    bool  ref_fs = false; // use_reference_cdef_fs: strengths predicted from the references, no search
    switch (level) {
    case 1: L = {16, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, 3, {1, 2, 3}, true, 1, 0}; break;
    case 2: L = {12, {0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14}, 3, {1, 2, 3}, false, 1, 0}; break;
    case 3: L = {8, {0, 2, 4, 6, 8, 10, 12, 14}, 3, {1, 2, 3}, true, 1, 0}; break;
    case 4: L = {5, {0, 4, 8, 12, 15}, 3, {1, 2, 3}, false, 1, 0}; break;
    case 5: L = {4, {0, 5, 10, 15}, 3, {1, 2, 3}, true, 1, 0}; break;
    case 6: L = {3, {0, 7, 15}, 3, {1, 2, 3}, false, 1, 0}; break;
    case 7: L = {3, {0, 7, 15}, 2, {1, 2}, true, 1, 0}; break;
    case 8: L = {3, {0, 7, 15}, 1, {2}, false, 1, 0}; break;
    case 9:
    case 10: L = {2, {0, 15}, 1, {2}, false, 4, 0}; break;
    case 12:
    case 13:
    case 16: L = {2, {0, 15}, 1, {2}, false, 4, 62}; break;
    case 11: L = {2, {0, 15}, 1, {2}, false, 4, 0}, ref_fs = true; break;
    case 14: L = {2, {0, 15}, 1, {2}, false, 4, 62}, ref_fs = true; break;
    case 15:
    case 17: L = {1, {0}, 0, {0}, false, 4, 62}, ref_fs = true; break;
    default: return SVTGPU_ERR_UNSUPPORTED; // 0: CDEF off
    }
    memset(c, 0, sizeof(*c));
    c->first_pass_fs_num          = (uint8_t)L.nfirst;
    c->default_second_pass_fs_num = (uint8_t)(L.nfirst * L.nsec);
    c->subsampling_factor         = L.ss;
    c->zero_fs_cost_bias          = L.bias;
    c->use_reference_cdef_fs      = ref_fs;
    for (int i = 0, sf = 0; i < L.nfirst; i++) {
        const uint8_t p              = pf_gi[L.first[i]];
        c->default_first_pass_fs[i]    = p;
        c->default_first_pass_fs_uv[i] = (int8_t)p;
        for (int j = 0; j < L.nsec; j++, sf++) {
            c->default_second_pass_fs[sf]    = (uint8_t)(p + L.sec[j]);
            c->default_second_pass_fs_uv[sf] = L.sec_uv ? (int8_t)(p + L.sec[j]) : (int8_t)-1;
        }
    }
    return SVTGPU_OK;
}

static int valid_controls(const SvtGpuCdefControls *c) {
    if (c->use_reference_cdef_fs)
        return c->pred_y_f >= 0 && c->pred_uv_f >= 0 && (c->subsampling_factor == 1 || c->subsampling_factor == 2 ||
                                                         c->subsampling_factor == 4);
    const int n = c->first_pass_fs_num + c->default_second_pass_fs_num;
    if (n <= 0 || n > 64)
        return 0;
    if (c->subsampling_factor != 1 && c->subsampling_factor != 2 && c->subsampling_factor != 4)
        return 0;
    for (int i = 0; i < n; i++) {
        const int code = i < c->first_pass_fs_num ? c->default_first_pass_fs[i]
                                                  : c->default_second_pass_fs[i - c->first_pass_fs_num];
        if (code > 63)
            return 0;
    }
    return 1;
}

static void build_table(const SvtGpuCdefControls *c, CdefStrengthTable *t) {
    memset(t, 0, sizeof(*t));
    for (int g = 0; g < 2; g++)
        for (int i = 0; i < 16; i++)
            for (int q = 0; q < 4; q++) t->luma[g].gi[i][q] = t->chroma[g].gi[i][q] = -1;
    const int nf = c->first_pass_fs_num;
    t->nstr      = nf + c->default_second_pass_fs_num;
    int first_of[64];
    for (int i = 0; i < 64; i++) first_of[i] = -1;
    auto add = [](CdefGroupTable &G, int level, int sc, int gi) {
        int li = 0;
        while (li < G.nlv && G.lv[li] != level) li++;
        if (li == G.nlv) G.lv[G.nlv++] = level;
        G.gi[li][sc] = gi;
        if (sc) G.sec_used |= 1 << sc;
    };
    for (int gi = 0; gi < t->nstr; gi++) {
        const bool first = gi < nf;
        const int  code  = first ? c->default_first_pass_fs[gi] : c->default_second_pass_fs[gi - nf];
        const bool uv    = first ? c->default_first_pass_fs_uv[gi] != -1 : c->default_second_pass_fs_uv[gi - nf] != -1;
        t->uv_on[gi]     = uv;
        t->alias[gi]     = (int8_t)first_of[code];
        if (first_of[code] >= 0) continue; // same code searched twice: copy its result
        first_of[code] = gi;
        const int level = code >> 2, sc = code & 3, g = level != 0;
        add(t->luma[g], level, sc, gi);
        if (uv) add(t->chroma[g], level, sc, gi);
    }
}

extern "C" int svtgpu_cdef_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuCdefFrameState **out) {
    if (!ctx || !out || width <= 0 || height <= 0 || (width & 7) || (height & 7))
        return SVTGPU_ERR_INVALID_ARG;
    auto *s      = new SvtGpuCdefFrameState{};
    s->ctx       = ctx;
    s->width     = width;
    s->height    = height;
    s->geo       = frame_geo(width, height);
    s->nfb       = s->geo.nvfb * s->geo.nhfb;
    s->mask_all  = 1;
    s->pick_settle = 24; // the first pick checks after step 24 (then after the previous pick's settling step)
    s->pick_parts = 64;
    const size_t nfb = s->nfb;
    bool ok = hipMalloc(&s->d_mask, (size_t)s->geo.b8_rows * s->geo.b8_cols) == hipSuccess &&
              hipMalloc(&s->d_mse, nfb * 2 * 64 * 8) == hipSuccess && hipMalloc(&s->d_skip, (nfb + 7) & ~(size_t)7) == hipSuccess &&
              hipMalloc(&s->d_dir, nfb * 64) == hipSuccess && hipMalloc(&s->d_var, nfb * 64 * 4) == hipSuccess &&
              hipMalloc(&s->d_fb_strength, nfb) == hipSuccess &&
              hipMalloc(&s->d_pick_part, (nfb * 128 + (size_t)3 * 4 * 4096 + 41 * 4 + (size_t)nfb * 64) * 8) == hipSuccess &&
              hipMalloc(&s->d_pick_out, 8 * 8) == hipSuccess && hipMalloc(&s->d_pick_lev, (size_t)(41 * 4 * 32 + 4 * 32 + 64) * 4) == hipSuccess &&
              hipMalloc(&s->d_fb_list, (2 * nfb + 1) * 4) == hipSuccess &&
              hipMalloc(&s->d_pick_xch, SVTGPU_PICK_XCH_BYTES) == hipSuccess &&
              hipMalloc(&s->d_apick, 64) == hipSuccess &&
              hipHostMalloc((void **)&s->h_pick, 512 + nfb, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
              hipHostGetDevicePointer((void **)&s->h_pick_dev, s->h_pick, 0) == hipSuccess;
    if (!ok) {
        svtgpu_cdef_state_destroy(s);
        return SVTGPU_ERR_OOM;
    }
    HIP_TRY(hipMemset(s->d_fb_strength, 0, nfb));
    HIP_TRY(hipMemset(s->d_apick, 0, 64));
    std::memset(s->h_pick, 0, 512 + nfb); // no record carries a sequence number yet
    HIP_TRY(hipMemset(s->d_pick_xch, 0, SVTGPU_PICK_XCH_BYTES)); // no word carries a valid tag
    HIP_TRY(hipMemset(s->d_skip, 0, (nfb + 7) & ~(size_t)7)); // the padding stays 0 (the tables' word sums)
    HIP_TRY(hipMemset(s->d_skip, 1, nfb));
    // the memsets above run on the null stream: done before any call on the caller's (non-blocking) streams, whose
    // first search may clear these tables
    HIP_TRY(hipStreamSynchronize(nullptr));
    s->own_mse      = s->d_mse;
    s->own_skip     = s->d_skip;
    s->own_dir      = s->d_dir;
    s->own_var      = s->d_var;
    s->fb_rect[0] = s->fb_rect[1] = 0, s->fb_rect[2] = s->geo.nhfb, s->fb_rect[3] = s->geo.nvfb;
    s->out_rect[0] = s->out_rect[1] = 0, s->out_rect[2] = width, s->out_rect[3] = height;
    *out = s;
    return SVTGPU_OK;
}

extern "C" void svtgpu_cdef_state_destroy(SvtGpuCdefFrameState *s) {
    if (!s)
        return;
    delete[] s->h_fb_kind;
    void *bufs[] = {s->d_fb_kind, s->d_mse_rem, s->d_mask, s->own_mse ? s->own_mse : s->d_mse, s->own_skip ? s->own_skip : s->d_skip,
                    s->own_dir ? s->own_dir : s->d_dir, s->own_var ? (void *)s->own_var : (void *)s->d_var, s->d_fb_strength, s->d_pick_part,
                    s->d_pick_out, s->d_pick_lev, s->d_fb_list, s->d_pick_xch, s->d_apick};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (s->h_pick) (void)hipHostFree(s->h_pick);
    svtgpu_prio_destroy(&s->prio);
    delete s;
}

extern "C" int svtgpu_cdef_set_fb_rows(SvtGpuCdefFrameState *s, int32_t fb_row_begin, int32_t fb_row_end) {
    if (!s || fb_row_begin < 0 || fb_row_end > s->geo.nvfb || fb_row_begin >= fb_row_end)
        return SVTGPU_ERR_INVALID_ARG;
    s->fb_rect[0] = 0, s->fb_rect[1] = fb_row_begin, s->fb_rect[2] = s->geo.nhfb, s->fb_rect[3] = fb_row_end;
    s->out_rect[0] = 0, s->out_rect[1] = fb_row_begin * 64, s->out_rect[2] = s->width;
    s->out_rect[3] = std::min(s->height, fb_row_end * 64);
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_set_tile(SvtGpuCdefFrameState *s, const int32_t fb_rect[4], const int32_t out_rect[4],
                                    SvtGpuComm *comm) {
    if (!s) return SVTGPU_ERR_INVALID_ARG;
    const int32_t all_fb[4] = {0, 0, s->geo.nhfb, s->geo.nvfb}, all_px[4] = {0, 0, s->width, s->height};
    const int32_t *f = fb_rect ? fb_rect : all_fb, *o = out_rect ? out_rect : all_px;
    if (f[0] < 0 || f[1] < 0 || f[2] > s->geo.nhfb || f[3] > s->geo.nvfb || f[0] >= f[2] || f[1] >= f[3] ||
        o[0] < 0 || o[1] < 0 || o[2] > s->width || o[3] > s->height || o[0] >= o[2] || o[1] >= o[3] ||
        ((o[0] | o[1] | o[2] | o[3]) & 1))
        return SVTGPU_ERR_INVALID_ARG;
    if (s->d_fb_kind && ((f[0] | f[1]) & 1)) return SVTGPU_ERR_INVALID_ARG; // SB128 areas are never cut
    std::memcpy(s->fb_rect, f, sizeof s->fb_rect);
    std::memcpy(s->out_rect, o, sizeof s->out_rect);
    s->comm     = comm;
    s->gathered = 0; // another comm or tile: the tables hold this rank's blocks only until the next pick sums them
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_bind_tables(SvtGpuCdefFrameState *s, void *mse_dev, void *skip_dev) {
    if (!s || (!mse_dev) != (!skip_dev))
        return SVTGPU_ERR_INVALID_ARG;
    s->d_mse  = mse_dev ? (uint64_t *)mse_dev : s->own_mse;
    s->d_skip = skip_dev ? (uint8_t *)skip_dev : s->own_skip;
    s->gathered = 0; // freshly bound tables are this rank's until the next pick sums them
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_bind_dir_tables(SvtGpuCdefFrameState *s, void *dir_dev, void *var_dev) {
    if (!s || (!dir_dev) != (!var_dev))
        return SVTGPU_ERR_INVALID_ARG;
    s->d_dir = dir_dev ? (uint8_t *)dir_dev : s->own_dir;
    s->d_var = var_dev ? (int32_t *)var_dev : s->own_var;
    s->gathered = 0;
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_clear_tables(SvtGpuCdefFrameState *s, void *stream) {
    if (!s)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(s->ctx, stream);
    // exactly nfb skip bytes: a bound skip table is [nfb] (svtgpu.h); the state's own copy keeps its zero padding
    HIP_TRY(hipMemsetAsync(s->d_mse, 0, (size_t)s->nfb * 2 * 64 * 8, st));
    HIP_TRY(hipMemsetAsync(s->d_skip, 0, (size_t)s->nfb, st));
    HIP_TRY(hipMemsetAsync(s->d_dir, 0, (size_t)s->nfb * 64, st));
    HIP_TRY(hipMemsetAsync(s->d_var, 0, (size_t)s->nfb * 64 * 4, st));
    s->gathered = 0;
    return SVTGPU_OK;
}

extern "C" int32_t svtgpu_cdef_state_nfb(const SvtGpuCdefFrameState *s) { return s ? s->nfb : -1; }

extern "C" int svtgpu_cdef_set_block_mask(SvtGpuCdefFrameState *s, const uint8_t *host_mask, void *stream) {
    if (!s)
        return SVTGPU_ERR_INVALID_ARG;
    if (!host_mask) {
        s->mask_all = 1;
        return SVTGPU_OK;
    }
    s->mask_all = 0;
    svtgpu_count_xfer(0, (size_t)s->geo.b8_rows * s->geo.b8_cols);
    HIP_TRY(hipMemcpyAsync(s->d_mask, host_mask, (size_t)s->geo.b8_rows * s->geo.b8_cols, hipMemcpyHostToDevice,
                           pick_stream(s->ctx, stream)));
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_set_fb_bsize(SvtGpuCdefFrameState *s, const uint8_t *fb_bsize, void *stream) {
    if (!s)
        return SVTGPU_ERR_INVALID_ARG;
    if (!fb_bsize) {
        if (s->d_fb_kind) (void)hipFree(s->d_fb_kind);
        if (s->d_mse_rem) (void)hipFree(s->d_mse_rem);
        delete[] s->h_fb_kind;
        s->d_fb_kind = nullptr, s->h_fb_kind = nullptr, s->d_mse_rem = nullptr;
        return SVTGPU_OK;
    }
    if (!s->h_fb_kind) { // all three buffers or none: the search folds SB128 areas only when d_fb_kind is set
        int8_t  *dk = nullptr;
        uint8_t *dr = nullptr;
        hipError_t e = hipMalloc(&dk, s->nfb);
        if (e == hipSuccess) e = hipMalloc(&dr, (size_t)3 * s->nfb * 64);
        if (e != hipSuccess) {
            if (dk) (void)hipFree(dk);
            svtgpu_set_last_hip_error(e, "cdef sb128 tables", __FILE__, __LINE__);
            return e == hipErrorOutOfMemory ? SVTGPU_ERR_OOM : SVTGPU_ERR_HIP;
        }
        s->d_fb_kind = dk, s->d_mse_rem = dr, s->h_fb_kind = new int8_t[s->nfb];
    }
    // BLOCK_64X128 = 13, BLOCK_128X64 = 14, BLOCK_128X128 = 15 (EbDefinitions.h); the parity tests of
    // EbCdefProcess.c:193-196 mark the halves the search skips
    const int nhfb = s->geo.nhfb;
    for (int f = 0; f < s->nfb; f++) {
        const int b = fb_bsize[f], fbr = f / nhfb, fbc = f - fbr * nhfb;
        int8_t    k = 0;
        if (((fbc & 1) && (b == 15 || b == 14)) || ((fbr & 1) && (b == 15 || b == 13)))
            k = -1;
        else if (b == 15 || b == 14 || b == 13)
            k = (int8_t)(b == 15 ? 1 : b == 14 ? 2 : 3);
        s->h_fb_kind[f] = k;
    }
    svtgpu_count_xfer(0, s->nfb);
    HIP_TRY(hipMemcpyAsync(s->d_fb_kind, s->h_fb_kind, s->nfb, hipMemcpyHostToDevice, pick_stream(s->ctx, stream)));
    HIP_TRY(hipStreamSynchronize(pick_stream(s->ctx, stream))); // the host array may be reused at once
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_search_frame(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                        const SvtGpuCdefControls *ctrls, int32_t base_q_idx, void *stream) {
    if (!s || !recon || !source || !ctrls || !valid_controls(ctrls))
        return SVTGPU_ERR_INVALID_ARG;
    if (recon->width != s->width || recon->height != s->height || source->width != s->width ||
        source->height != s->height || recon->bit_depth != source->bit_depth)
        return SVTGPU_ERR_INVALID_ARG;
    if (base_q_idx < 0 || base_q_idx > 255)
        return SVTGPU_ERR_INVALID_ARG;
    CdefStrengthTable tab;
    hipStream_t       st = pick_stream(s->ctx, stream);
    // tiled over GPUs: zeros outside this rank's filter blocks, so the pick's word sums over the ranks gather the tables
    if (svtgpu_comm_tiled(s->comm))
        if (int rc = svtgpu_cdef_clear_tables(s, st)) return rc;
    s->gathered = 0; // this rank's blocks only until the next pick sums them
    if (ctrls->use_reference_cdef_fs) { // directions / variances only: an empty strength table
        memset(&tab, 0, sizeof(tab));
        return svtgpu_launch_cdef_search(s, recon, source, &tab, ctrls->subsampling_factor, 3 + (base_q_idx >> 6), st);
    }
    build_table(ctrls, &tab);
    if (int rc = svtgpu_launch_cdef_search(s, recon, source, &tab, ctrls->subsampling_factor, 3 + (base_q_idx >> 6), st))
        return rc;
    if (!s->d_fb_kind)
        return SVTGPU_OK;
    unsigned long long uv_on = 0;
    for (int gi = 0; gi < 64; gi++) // entries past the searched strengths are zero sums, like tested ones
        uv_on |= (unsigned long long)(gi >= tab.nstr || tab.uv_on[gi] != 0) << gi;
    return svtgpu_launch_cdef_sb128_fold(s, uv_on, recon->bit_depth - 8, ctrls->subsampling_factor, st);
}

// the pick of svtgpu_cdef_pick (params_out) and svtgpu_cdef_pick_async (params_out == nullptr: no host wait)
static int cdef_pick_common(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                            uint64_t lambda, SvtGpuCdefParams *params_out, int8_t *fb_strength_out, hipStream_t st) {
    const bool async_ = params_out == nullptr;
    // the ranks' search tables (zero elsewhere) summed = gathered; once per search, so a second pick on the same
    // search (another level, another lambda) reads the gathered tables instead of summing them again
    if (svtgpu_comm_tiled(s->comm) && !s->gathered) {
        const size_t nfb = s->nfb;
        if (int rc = svtgpu_comm_sum(s->comm, s->d_dir, nfb * 64 / 8, true, st, SVTGPU_XCH_CDEF)) return rc;
        if (int rc = svtgpu_comm_sum(s->comm, s->d_var, nfb * 64 * 4 / 8, true, st, SVTGPU_XCH_CDEF)) return rc;
        if (!ctrls->use_reference_cdef_fs) {
            if (int rc = svtgpu_comm_sum(s->comm, s->d_mse, nfb * 2 * 64, true, st, SVTGPU_XCH_CDEF)) return rc;
            // word sums over the state's padded copy: a bound table is exactly [nfb] bytes
            const size_t words = (nfb + 7) / 8;
            if (s->d_skip != s->own_skip) HIP_TRY(hipMemcpyAsync(s->own_skip, s->d_skip, nfb, hipMemcpyDeviceToDevice, st));
            if (int rc = svtgpu_comm_sum(s->comm, s->own_skip, words, true, st, SVTGPU_XCH_CDEF)) return rc;
            if (s->d_skip != s->own_skip) HIP_TRY(hipMemcpyAsync(s->d_skip, s->own_skip, nfb, hipMemcpyDeviceToDevice, st));
        }
        s->gathered = 1;
    }
    if (async_) s->apick_ref = ctrls->use_reference_cdef_fs != 0, s->apick_pending = 1, s->apick_ready = 1;
    if (ctrls->use_reference_cdef_fs) { // EbEncCdef.c:744-789: index 0 for every filter block, one pair
        SvtGpuCdefParams q;
        memset(&q, 0, sizeof(q));
        q.cdef_damping        = (uint8_t)(3 + (base_q_idx >> 6));
        q.cdef_bits           = 0;
        q.cdef_y_strength[0]  = (uint8_t)ctrls->pred_y_f;
        q.cdef_uv_strength[0] = (uint8_t)ctrls->pred_uv_f;
        HIP_TRY(hipMemsetAsync(s->d_fb_strength, 0, s->nfb, st));
        if (async_) { // the apply's device copy, in stream order
            s->apick_params = q;
            return svtgpu_launch_cdef_set_params(s, &q, st);
        }
        *params_out = q;
        if (fb_strength_out) memset(fb_strength_out, 0, s->nfb);
        // tiled: the dir / var exchanges above are bounded here, not by some later unbounded wait
        if (svtgpu_comm_tiled(s->comm)) return svtgpu_comm_wait(s->comm, st);
        return SVTGPU_OK;
    }
    hipStream_t hs;
    if (int rc = svtgpu_prio_enter(&s->prio, st, &hs)) return rc;
    if (int rc = svtgpu_cdef_pick_impl(s, ctrls, base_q_idx, lambda, params_out, fb_strength_out, hs)) {
        (void)svtgpu_prio_leave(&s->prio, hs, st);
        return rc;
    }
    if (s->d_fb_kind) { // the halves of 128-wide areas take the area's index (EbEncCdef.c:893-909)
        if (int rc = svtgpu_launch_cdef_sb128_dup(s, hs)) {
            (void)svtgpu_prio_leave(&s->prio, hs, st);
            return rc;
        }
        if (fb_strength_out) svtgpu_cdef_sb128_dup_host(s, fb_strength_out);
    }
    return svtgpu_prio_leave(&s->prio, hs, st);
}

extern "C" int svtgpu_cdef_pick(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                                uint64_t lambda, SvtGpuCdefParams *params_out, int8_t *fb_strength_out, void *stream) {
    if (!s || !ctrls || !params_out || !valid_controls(ctrls))
        return SVTGPU_ERR_INVALID_ARG;
    return cdef_pick_common(s, ctrls, base_q_idx, lambda, params_out, fb_strength_out, pick_stream(s->ctx, stream));
}

// The pick with no host wait: everything in stream order, the frame parameters left in device memory for
// svtgpu_cdef_apply_frame(params = NULL); svtgpu_cdef_read_params returns them (and the per-FB strengths) later.
extern "C" int svtgpu_cdef_pick_async(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                                      uint64_t lambda, void *stream) {
    if (!s || !ctrls || !valid_controls(ctrls))
        return SVTGPU_ERR_INVALID_ARG;
    return cdef_pick_common(s, ctrls, base_q_idx, lambda, nullptr, nullptr, pick_stream(s->ctx, stream));
}

extern "C" int svtgpu_cdef_read_params(SvtGpuCdefFrameState *s, SvtGpuCdefParams *params_out, int8_t *fb_strength_out,
                                       void *stream) {
    if (!s || !params_out || !s->apick_ready)
        return SVTGPU_ERR_INVALID_ARG;
    if (int rc = svtgpu_cdef_pick_read(s, params_out, fb_strength_out, pick_stream(s->ctx, stream))) return rc;
    if (fb_strength_out && s->d_fb_kind && !s->apick_ref) svtgpu_cdef_sb128_dup_host(s, fb_strength_out);
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_set_fb_strength(SvtGpuCdefFrameState *s, const int8_t *fb_strength, void *stream) {
    if (!s || !fb_strength)
        return SVTGPU_ERR_INVALID_ARG;
    svtgpu_count_xfer(0, s->nfb);
    HIP_TRY(hipMemcpyAsync(s->d_fb_strength, fb_strength, s->nfb, hipMemcpyHostToDevice, pick_stream(s->ctx, stream)));
    return SVTGPU_OK;
}

extern "C" int svtgpu_cdef_apply_frame(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, SvtGpuFrame *out,
                                       const SvtGpuCdefParams *params, void *stream) {
    if (!s || !recon || !out || recon == out || (!params && !s->apick_ready))
        return SVTGPU_ERR_INVALID_ARG; // params == NULL: the last svtgpu_cdef_pick_async's, from device memory
    if (recon->width != s->width || recon->height != s->height || out->width != s->width ||
        out->height != s->height || out->bit_depth != recon->bit_depth)
        return SVTGPU_ERR_INVALID_ARG;
    if (params && params->cdef_bits > 3)
        return SVTGPU_ERR_INVALID_ARG;
    for (int i = 0; params && i < (1 << params->cdef_bits); i++)
        if (params->cdef_y_strength[i] > 63 || params->cdef_uv_strength[i] > 63)
            return SVTGPU_ERR_INVALID_ARG;
    return svtgpu_launch_cdef_apply(s, recon, out, params, pick_stream(s->ctx, stream));
}

extern "C" int svtgpu_cdef_read_state(SvtGpuCdefFrameState *s, uint64_t *mse, uint8_t *skip, uint8_t *dir,
                                      int32_t *var, void *stream) {
    if (!s)
        return SVTGPU_ERR_INVALID_ARG;
    hipStream_t  st  = pick_stream(s->ctx, stream);
    const size_t nfb = s->nfb;
    svtgpu_count_xfer(1, (mse ? nfb * 2 * 64 * 8 : 0) + (skip ? nfb : 0) + (dir ? nfb * 64 : 0) + (var ? nfb * 64 * 4 : 0));
    if (mse) HIP_TRY(hipMemcpyAsync(mse, s->d_mse, nfb * 2 * 64 * 8, hipMemcpyDeviceToHost, st));
    if (skip) HIP_TRY(hipMemcpyAsync(skip, s->d_skip, nfb, hipMemcpyDeviceToHost, st));
    if (dir) HIP_TRY(hipMemcpyAsync(dir, s->d_dir, nfb * 64, hipMemcpyDeviceToHost, st));
    if (var) HIP_TRY(hipMemcpyAsync(var, s->d_var, nfb * 64 * 4, hipMemcpyDeviceToHost, st));
    return svtgpu_comm_wait(s->comm, st); // bounded when the tables' exchange sits before the copies
    return SVTGPU_OK;
}

extern "C" void *svtgpu_cdef_mse_device_ptr(SvtGpuCdefFrameState *s) { return s ? (void *)s->d_mse : nullptr; }
