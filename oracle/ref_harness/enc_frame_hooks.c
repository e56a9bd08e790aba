/*
 * enc_frame_hooks.c — libsvtgpu's frame-level entry points inside the reference encoder (test infrastructure; the
 * `frame` mode of enc_drop_in, tests/test_encoder_drop_in.py).
 *
 * The encoder's process bodies call their frame-level filter functions across translation units of libsvtenc.so,
 * through the PLT.  This file defines the same symbols in the executable, so ELF symbol interposition binds the
 * library's calls here (no reference source is edited or copied):
 *   svt_aom_dlf_kernel   (EbDlfProcess.c:96-106):  svt_av1_pick_filter_level(FULL_IMAGE) -> svtgpu_dlf_pick,
 *                                                  svt_av1_loop_filter_frame              -> svtgpu_dlf_frame;
 *   svt_aom_cdef_kernel  (EbCdefProcess.c:509-515): finish_cdef_search -> svtgpu_cdef_search_frame + svtgpu_cdef_pick
 *                                                  (the whole-frame device search; the process body's own per-segment
 *                                                  cdef_seg_search is static and still runs, its tables unused),
 *                                                  svt_av1_cdef_frame -> svtgpu_cdef_apply_frame;
 *   svt_aom_rest_kernel  (EbRestProcess.c:580-626): restoration_seg_search -> nothing (the device searches the frame),
 *                                                  rest_finish_search -> svtgpu_lr_search_frame + svtgpu_lr_finish_frame,
 *                                                  svt_av1_loop_restoration_filter_frame -> svtgpu_lr_apply_frame;
 *   the CCSO calls of the CDEF process body (EbCdefProcess.c:621-623, live only in the ccso build of the encoder,
 *   oracle/ref_harness/with_ccso.py): ccso_search -> svtgpu_ccso_search_frame, ccso_frame -> svtgpu_ccso_apply_plane.
 * Each hook moves the encoder's picture buffers to the device (svtgpu_frame_upload) and its results back into the
 * encoder's own structures exactly where the reference function writes them (frame header fields, mode-info grid,
 * restoration units, the recon samples).  Configurations the library does not cover (DLF methods other than
 * FULL_IMAGE, delta LF, superres / resize, the previous-frame Wiener coefficients, the reference-based SGR ep range)
 * call the encoder's own function (dlsym RTLD_NEXT) and count a fallback.  A picture whose size is off the 8-sample
 * grid runs on the device too: the deblocking / CDEF frames are the encoder's padded (8-aligned) pictures, the loop
 * restoration state the crop size frm_size.frame_width x frame_height (EbPictureControlSet.c:1207).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbPictureControlSet.h"
#include "EbSequenceControlSet.h"
#include "EbDeblockingFilter.h"
#include "EbRestoration.h"
#include "EbModeDecisionProcess.h"
#include "EbInterPrediction.h"
#include "aom_dsp_rtcd.h"
#include "common_dsp_rtcd.h"
#include "EbMcp.h"
#include "svtgpu_rtcd.h"
#include "EbCcso.h"

void    svt_aom_get_recon_pic(PictureControlSet *pcs, EbPictureBufferDesc **recon_ptr, Bool is_highbd);
int32_t svt_sb_all_skip(PictureControlSet *pcs, const Av1Common *const cm, int32_t mi_row, int32_t mi_col);

static int             g_on;
static uint64_t        g_calls, g_fallbacks;
/* device calls by kind: DLF pick, DLF filter, CDEF pick, CDEF apply, LR search, LR apply; and frames whose LR search
 * chose a filter for some plane (so the apply really filtered) */
enum { K_DLF_PICK, K_DLF_FRAME, K_CDEF_PICK, K_CDEF_APPLY, K_LR_SEARCH, K_LR_APPLY, K_LR_ON, K_CCSO_SEARCH,
       K_CCSO_APPLY, K_CCSO_ON, K_N };
static uint64_t g_kind[K_N];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static SvtGpuContext  *g_ctx;

void enc_frame_hooks_enable(int on) { g_on = on; }
/* ENC_HOOK_STAGES (diagnostics): the stages whose hooks are active, bits 1 DLF, 2 CDEF, 4 LR, 8 CCSO (default all) */
static int stage_on(int bit) {
    static int m = -1;
    if (m < 0) {
        const char *e = getenv("ENC_HOOK_STAGES");
        m             = e ? atoi(e) : 15;
    }
    return g_on && (m & bit);
}
uint64_t enc_frame_hook_calls(void) { return g_calls; }
uint64_t enc_frame_hook_fallbacks(void) { return g_fallbacks; }
void enc_frame_hook_kinds(uint64_t out[K_N]) { memcpy(out, g_kind, sizeof g_kind); }

static void die(const char *what, int rc) {
    fprintf(stderr, "enc_frame_hooks: %s failed (%d): %s\n", what, rc, svtgpu_error_string(rc));
    exit(6);
}
#define GPU(call)                              \
    do {                                       \
        int rc_ = (call);                      \
        if (rc_ != SVTGPU_OK) die(#call, rc_); \
    } while (0)

static void count_kind(int fallback, int kind) {
    pthread_mutex_lock(&g_mu);
    if (fallback) g_fallbacks++;
    else g_calls++, g_kind[kind]++;
    pthread_mutex_unlock(&g_mu);
}
#define count(fb) count_kind(fb, KIND)

/* ---- per-picture device state (the encoder runs several pictures through the stages at once) ---- */
typedef struct Ctx {
    PictureControlSet    *pcs;
    int                   w, h, bd; /* the coded (8-aligned) picture the frames hold */
    int                   cw, ch;   /* the crop size loop restoration covers */
    SvtGpuFrame          *R, *S, *D, *O, *L; /* recon in, source, deblocked (pre-CDEF), CDEF output, LR output */
    SvtGpuDlfState       *dlf;
    SvtGpuCdefFrameState *cdef;
    SvtGpuLrState        *lr;
    int32_t               lr_units[3];
    int                   d_valid, cdef_searched, lr_searched;
    int32_t               lr_ft[3];
    SvtGpuCcsoState      *ccso; /* the CCSO search / apply (the ccso build of the encoder only) */
    void                 *d_ext, *d_org[3], *d_rec[3], *d_pl[3];
    size_t                pl_bytes[3];
} Ctx;
static Ctx g_ctxs[64];

static Ctx *ctx_of(PictureControlSet *pcs) {
    pthread_mutex_lock(&g_mu);
    if (!g_ctx) GPU(svtgpu_context_create(0, &g_ctx));
    Ctx *c = NULL;
    for (int i = 0; i < 64 && !c; i++)
        if (g_ctxs[i].pcs == pcs) c = &g_ctxs[i];
    for (int i = 0; i < 64 && !c; i++)
        if (!g_ctxs[i].pcs) c = &g_ctxs[i], c->pcs = pcs;
    pthread_mutex_unlock(&g_mu);
    if (!c) die("ctx_of: more than 64 pictures in flight", -1);
    SequenceControlSet *scs = pcs->scs;
    Av1Common          *cm  = pcs->ppcs->av1_cm;
    const int cw = cm->frm_size.frame_width, ch = cm->frm_size.frame_height;
    const int w = (cw + 7) & ~7, h = (ch + 7) & ~7, bd = (int)scs->static_config.encoder_bit_depth;
    if (c->R && (c->cw != cw || c->ch != ch || c->bd != bd)) die("picture geometry changed", -1);
    if (!c->R) {
        c->w = w, c->h = h, c->cw = cw, c->ch = ch, c->bd = bd;
        SvtGpuFrame **f[5] = {&c->R, &c->S, &c->D, &c->O, &c->L};
        for (int i = 0; i < 5; i++) GPU(svtgpu_frame_create(g_ctx, w, h, bd, f[i]));
        GPU(svtgpu_dlf_state_create(g_ctx, w, h, &c->dlf));
        /* the unpadded size set_lpf_parameters stops at (EbDeblockingFilter.c:99-129, :173-178) */
        GPU(svtgpu_dlf_set_crop(c->dlf, scs->max_input_luma_width - scs->max_input_pad_right,
                                scs->max_input_luma_height - scs->max_input_pad_bottom));
        GPU(svtgpu_cdef_state_create(g_ctx, w, h, &c->cdef));
    }
    return c;
}

/* the visible-area origin and stride (samples) of each plane of an encoder picture buffer */
static void pic_planes(const EbPictureBufferDesc *p, int is16, void *pl[3], int32_t st[3]) {
    const int b = is16 ? 2 : 1;
    pl[0] = p->buffer_y + (size_t)(p->org_x + p->org_y * p->stride_y) * b;
    pl[1] = p->buffer_cb + (size_t)((p->org_x >> 1) + (p->org_y >> 1) * p->stride_cb) * b;
    pl[2] = p->buffer_cr + (size_t)((p->org_x >> 1) + (p->org_y >> 1) * p->stride_cr) * b;
    st[0] = p->stride_y, st[1] = p->stride_cb, st[2] = p->stride_cr;
}
static void upload_pic(SvtGpuFrame *f, const EbPictureBufferDesc *p, int is16, int p0, int p1) {
    void   *pl[3];
    int32_t st[3];
    pic_planes(p, is16, pl, st);
    for (int q = p0; q < p1; q++) GPU(svtgpu_frame_upload(f, q, pl[q], st[q], NULL));
}
static void download_pic(SvtGpuFrame *f, EbPictureBufferDesc *p, int is16, int p0, int p1) {
    void   *pl[3];
    int32_t st[3];
    pic_planes(p, is16, pl, st);
    for (int q = p0; q < p1; q++) GPU(svtgpu_frame_download(f, q, pl[q], st[q], NULL));
    GPU(svtgpu_synchronize(g_ctx, NULL));
}
/* Yv12BufferConfig planes (16-bit buffers are CONVERT_TO_BYTEPTR addresses) */
static void yv12_planes(const Yv12BufferConfig *y, int hbd, void *pl[3], int32_t st[3]) {
    uint8_t *b[3] = {y->y_buffer, y->u_buffer, y->v_buffer};
    for (int q = 0; q < 3; q++) pl[q] = hbd ? (void *)CONVERT_TO_SHORTPTR(b[q]) : (void *)b[q];
    st[0] = y->y_stride, st[1] = st[2] = y->uv_stride;
}

/* the library covers 4:2:0 pictures, 8/10-bit, without superres / resize; the encoder pads its pictures to the
 * 8-sample grid (aligned_width / _height) and the frame-level stages work on that padded size */
static int frame_supported(PictureControlSet *pcs) {
    SequenceControlSet *scs = pcs->scs;
    Av1Common          *cm  = pcs->ppcs->av1_cm;
    const int w = cm->frm_size.frame_width, h = cm->frm_size.frame_height, bd = (int)scs->static_config.encoder_bit_depth;
    return g_on && pcs->ppcs->aligned_width == ((w + 7) & ~7) && pcs->ppcs->aligned_height == ((h + 7) & ~7) &&
           (bd == 8 || bd == 10) &&
           scs->static_config.encoder_color_format == EB_YUV420 && scs->static_config.superres_mode == SUPERRES_NONE &&
           scs->static_config.resize_mode == RESIZE_NONE && cm->frm_size.superres_upscaled_width == w &&
           (scs->seq_header.sb_size == BLOCK_64X64 || scs->seq_header.sb_size == BLOCK_128X128);
}

/* The deblocked picture, before CDEF: the DLF process saves the restoration stripe boundaries from it
 * (EbDlfProcess.c:112-114, after_cdef = 0); the device LR apply reads those rows from this copy (D) instead */
typedef void (*SaveLinesFn)(const Yv12BufferConfig *, Av1Common *, int32_t);
void svt_av1_loop_restoration_save_boundary_lines(const Yv12BufferConfig *frame, Av1Common *cm, int32_t after_cdef) {
    static SaveLinesFn orig;
    if (!orig) orig = (SaveLinesFn)dlsym(RTLD_NEXT, "svt_av1_loop_restoration_save_boundary_lines");
    if (stage_on(4) && !after_cdef && frame_supported(cm->child_pcs)) {
        Ctx    *c = ctx_of(cm->child_pcs);
        void   *pl[3];
        int32_t st[3];
        yv12_planes(frame, cm->use_highbitdepth, pl, st);
        for (int q = 0; q < 3; q++) GPU(svtgpu_frame_upload(c->D, q, pl[q], st[q], NULL));
        GPU(svtgpu_synchronize(g_ctx, NULL));
        c->d_valid = 1;
    }
    orig(frame, cm, after_cdef); /* the encoder's own boundary buffers stay filled (any fallback apply reads them) */
}

/* ============================== deblocking ============================== */
static void lf_params(PictureControlSet *pcs, SvtGpuLfParams *p) {
    FrameHeader             *fh = &pcs->ppcs->frm_hdr;
    const struct LoopFilter *lf = &fh->loop_filter_params;
    memset(p, 0, sizeof *p);
    p->filter_level[0] = lf->filter_level[0], p->filter_level[1] = lf->filter_level[1];
    p->filter_level_u = lf->filter_level_u, p->filter_level_v = lf->filter_level_v;
    p->sharpness_level        = lf->sharpness_level;
    p->mode_ref_delta_enabled = lf->mode_ref_delta_enabled;
    for (int k = 0; k < 8; k++) p->ref_deltas[k] = lf->ref_deltas[k];
    for (int k = 0; k < 2; k++) p->mode_deltas[k] = lf->mode_deltas[k];
    p->segmentation_enabled = fh->segmentation_params.segmentation_enabled;
    for (int s = 0; s < 8; s++)
        for (int f = 0; f < 8; f++) {
            p->seg_feature_data[s][f]    = fh->segmentation_params.feature_data[s][f];
            p->seg_feature_enabled[s][f] = fh->segmentation_params.feature_enabled[s][f];
        }
}
static void set_mode_info(Ctx *c, PictureControlSet *pcs) {
    Av1Common *cm = pcs->ppcs->av1_cm;
    const int  mr = ((c->h + 7) & ~7) >> 2, mc = ((c->w + 7) & ~7) >> 2;
    SvtGpuLfMi *mi = calloc((size_t)mr * mc, sizeof *mi);
    for (int r = 0; r < mr; r++)
        for (int q = 0; q < mc; q++) {
            const BlockModeInfoEnc *b = &pcs->mi_grid_base[(size_t)r * cm->mi_stride + q]->mbmi.block_mi;
            SvtGpuLfMi          *m = &mi[(size_t)r * mc + q];
            m->bsize = (uint8_t)b->bsize, m->tx_depth = b->tx_depth, m->skip = b->skip;
            m->ref_frame0 = (int8_t)b->ref_frame[0], m->mode = (uint8_t)b->mode, m->segment_id = b->segment_id;
        }
    GPU(svtgpu_dlf_set_mode_info(c->dlf, mi, NULL));
    GPU(svtgpu_synchronize(g_ctx, NULL));
    free(mi);
}
static int dlf_supported(PictureControlSet *pcs) {
    return frame_supported(pcs) && !pcs->ppcs->frm_hdr.delta_lf_params.delta_lf_present;
}

typedef EbErrorType (*PickFn)(EbPictureBufferDesc *, PictureControlSet *, LpfPickMethod);
#undef KIND
#define KIND K_DLF_PICK
EbErrorType svt_av1_pick_filter_level(EbPictureBufferDesc *srcBuffer, PictureControlSet *pcs, LpfPickMethod method) {
    static PickFn orig;
    if (!orig) orig = (PickFn)dlsym(RTLD_NEXT, "svt_av1_pick_filter_level");
    if (!stage_on(1)) return orig(srcBuffer, pcs, method);
    if (method != LPF_PICK_FROM_FULL_IMAGE || !dlf_supported(pcs)) {
        count(1);
        return orig(srcBuffer, pcs, method);
    }
    count(0);
    SequenceControlSet      *scs  = pcs->scs;
    PictureParentControlSet *ppcs = pcs->ppcs;
    struct LoopFilter       *lf   = &ppcs->frm_hdr.loop_filter_params;
    lf->sharpness_level           = 0; /* EbDeblockingFilter.c:1136 */
    /* dlf_avg: the search starts from the references' average levels (:1172-1203) */
    if (ppcs->dlf_ctrls.dlf_avg && ppcs->tot_ref_frame_types > 0) {
        int32_t t0 = 0, t1 = 0, tu = 0, tv = 0, n = 0;
        for (uint32_t it = 0; it < ppcs->tot_ref_frame_types; ++it) {
            MvReferenceFrame rf[2];
            av1_set_ref_frame(rf, ppcs->ref_frame_type_arr[it]);
            if (rf[1] != NONE_FRAME) continue;
            const EbReferenceObject *ro =
                pcs->ref_pic_ptr_array[get_list_idx(rf[0])][get_ref_frame_idx(rf[0])]->object_ptr;
            t0 += ro->filter_level[0], t1 += ro->filter_level[1], tu += ro->filter_level_u, tv += ro->filter_level_v;
            n++;
        }
        lf->filter_level[0] = t0 / n, lf->filter_level[1] = t1 / n, lf->filter_level_u = tu / n;
        lf->filter_level_v = tv / n;
    }
    Ctx *c = ctx_of(pcs);
    const int is16 = scs->is_16bit_pipeline;
    EbPictureBufferDesc *recon;
    svt_aom_get_recon_pic(pcs, &recon, is16);
    upload_pic(c->R, recon, is16, 0, 3);
    upload_pic(c->S, is16 ? pcs->input_frame16bit : ppcs->enhanced_pic, is16, 0, 3);
    set_mode_info(c, pcs);
    SvtGpuLfParams p;
    lf_params(pcs, &p);
    GPU(svtgpu_dlf_pick(c->dlf, c->R, c->S, &p, ppcs->dlf_ctrls.dlf_avg, ppcs->dlf_ctrls.dlf_avg_uv,
                        pcs->temporal_layer_index, ppcs->dlf_ctrls.early_exit_convergence,
                        ppcs->frm_hdr.tx_mode == ONLY_4X4, NULL));
    lf->filter_level[0] = p.filter_level[0], lf->filter_level[1] = p.filter_level[1];
    lf->filter_level_u = p.filter_level_u, lf->filter_level_v = p.filter_level_v;
    return EB_ErrorNone;
}

typedef void (*LfFrameFn)(EbPictureBufferDesc *, PictureControlSet *, int32_t, int32_t);
#undef KIND
#define KIND K_DLF_FRAME
void svt_av1_loop_filter_frame(EbPictureBufferDesc *frame_buffer, PictureControlSet *pcs, int32_t plane_start,
                               int32_t plane_end) {
    static LfFrameFn orig;
    if (!orig) orig = (LfFrameFn)dlsym(RTLD_NEXT, "svt_av1_loop_filter_frame");
    if (!stage_on(1)) return orig(frame_buffer, pcs, plane_start, plane_end);
    if (!dlf_supported(pcs)) {
        count(1);
        return orig(frame_buffer, pcs, plane_start, plane_end);
    }
    count(0);
    Ctx      *c    = ctx_of(pcs);
    const int is16 = pcs->scs->is_16bit_pipeline;
    upload_pic(c->R, frame_buffer, is16, plane_start, plane_end);
    set_mode_info(c, pcs);
    SvtGpuLfParams p;
    lf_params(pcs, &p);
    GPU(svtgpu_dlf_frame(c->dlf, c->R, &p, plane_start, plane_end, NULL));
    download_pic(c->R, frame_buffer, is16, plane_start, plane_end);
}

/* ================================= CDEF ================================= */
static void cdef_controls(const CdefControls *cc, SvtGpuCdefControls *g) {
    memset(g, 0, sizeof *g);
    g->first_pass_fs_num          = cc->first_pass_fs_num;
    g->default_second_pass_fs_num = cc->default_second_pass_fs_num;
    memcpy(g->default_first_pass_fs, cc->default_first_pass_fs, sizeof g->default_first_pass_fs);
    memcpy(g->default_second_pass_fs, cc->default_second_pass_fs, sizeof g->default_second_pass_fs);
    memcpy(g->default_first_pass_fs_uv, cc->default_first_pass_fs_uv, sizeof g->default_first_pass_fs_uv);
    memcpy(g->default_second_pass_fs_uv, cc->default_second_pass_fs_uv, sizeof g->default_second_pass_fs_uv);
    g->subsampling_factor    = cc->subsampling_factor;
    g->zero_fs_cost_bias     = cc->zero_fs_cost_bias;
    g->use_reference_cdef_fs = cc->use_reference_cdef_fs;
    g->pred_y_f              = cc->pred_y_f;
    g->pred_uv_f             = cc->pred_uv_f;
}

typedef void (*FinishFn)(PictureControlSet *);
#undef KIND
#define KIND K_CDEF_PICK
void finish_cdef_search(PictureControlSet *pcs) {
    static FinishFn orig;
    if (!orig) orig = (FinishFn)dlsym(RTLD_NEXT, "finish_cdef_search");
    if (!stage_on(2)) return orig(pcs);
    if (!frame_supported(pcs)) {
        count(1);
        return orig(pcs);
    }
    count(0);
    SequenceControlSet      *scs  = pcs->scs;
    PictureParentControlSet *ppcs = pcs->ppcs;
    FrameHeader             *fh   = &ppcs->frm_hdr;
    Av1Common               *cm   = ppcs->av1_cm;
    Ctx                     *c    = ctx_of(pcs);
    const int                is16 = scs->is_16bit_pipeline;
    /* the DLF output (pcs->cdef_input_recon, EbDlfProcess.c:117-127) and the source */
    EbPictureBufferDesc *recon;
    svt_aom_get_recon_pic(pcs, &recon, is16);
    upload_pic(c->D, recon, is16, 0, 3);
    upload_pic(c->S, is16 ? pcs->input_frame16bit : ppcs->enhanced_pic, is16, 0, 3);
    /* the 8x8 blocks svt_sb_compute_cdef_list lists (any of the four mi non-skip) and the SB128 areas */
    const int mr = cm->mi_rows, mc = cm->mi_cols, b8r = mr >> 1, b8c = mc >> 1;
    uint8_t  *mask = malloc((size_t)b8r * b8c);
    for (int r = 0; r < b8r; r++)
        for (int q = 0; q < b8c; q++) {
            int all = 1;
            for (int dr = 0; dr < 2; dr++)
                for (int dq = 0; dq < 2; dq++)
                    all &= pcs->mi_grid_base[(size_t)(2 * r + dr) * cm->mi_stride + 2 * q + dq]->mbmi.block_mi.skip != 0;
            mask[(size_t)r * b8c + q] = (uint8_t)!all;
        }
    GPU(svtgpu_cdef_set_block_mask(c->cdef, mask, NULL));
    const int nvfb = (mr + 15) / 16, nhfb = (mc + 15) / 16, nfb = nvfb * nhfb;
    uint8_t  *fbb  = malloc((size_t)nfb);
    for (int f = 0; f < nfb; f++)
        fbb[f] = (uint8_t)pcs->mi_grid_base[(size_t)16 * (f / nhfb) * cm->mi_stride + 16 * (f % nhfb)]->mbmi.block_mi.bsize;
    GPU(svtgpu_cdef_set_fb_bsize(c->cdef, scs->seq_header.sb_size == BLOCK_128X128 ? fbb : NULL, NULL));
    SvtGpuCdefControls gc;
    cdef_controls(&ppcs->cdef_ctrls, &gc);
    const int q = fh->quantization_params.base_q_idx;
    GPU(svtgpu_cdef_search_frame(c->cdef, c->D, c->S, &gc, q, NULL));
    uint32_t fast_lambda = 0, full_lambda = 0; /* EbEncCdef.c:807-814 */
    (*svt_aom_av1_lambda_assignment_function_table[ppcs->pred_structure])(
        pcs, &fast_lambda, &full_lambda, (uint8_t)ppcs->enhanced_pic->bit_depth, (uint8_t)q, FALSE);
    SvtGpuCdefParams prm;
    int8_t          *fbs = malloc((size_t)nfb);
    GPU(svtgpu_cdef_pick(c->cdef, &gc, q, full_lambda, &prm, fbs, NULL));
    uint8_t *skip = malloc((size_t)nfb);
    GPU(svtgpu_cdef_read_state(c->cdef, NULL, skip, NULL, NULL, NULL));
    /* the frame header and the per-FB indices where finish_cdef_search writes them (EbEncCdef.c:874-926) */
    fh->cdef_params.cdef_bits    = prm.cdef_bits;
    fh->cdef_params.cdef_damping = prm.cdef_damping;
    ppcs->nb_cdef_strengths      = 1 << prm.cdef_bits;
    for (int j = 0; j < ppcs->nb_cdef_strengths; j++)
        fh->cdef_params.cdef_y_strength[j] = prm.cdef_y_strength[j],
        fh->cdef_params.cdef_uv_strength[j] = prm.cdef_uv_strength[j];
    for (int f = 0; f < nfb; f++) {
        const int fbr = f / nhfb, fbc = f % nhfb;
        const int idx = 16 * fbr * pcs->mi_stride + 16 * fbc;
        const BlockSize bs = pcs->mi_grid_base[idx]->mbmi.block_mi.bsize;
        if (((fbc & 1) && (bs == BLOCK_128X128 || bs == BLOCK_128X64)) ||
            ((fbr & 1) && (bs == BLOCK_128X128 || bs == BLOCK_64X128)))
            continue; /* the second half of a 128-wide area */
        if (gc.use_reference_cdef_fs ? svt_sb_all_skip(pcs, cm, fbr * 16, fbc * 16) : skip[f]) continue;
        const int8_t g = fbs[f];
        pcs->mi_grid_base[idx]->mbmi.cdef_strength = g;
        if (bs == BLOCK_128X128 || bs == BLOCK_128X64) pcs->mi_grid_base[idx + 16]->mbmi.cdef_strength = g;
        if (bs == BLOCK_128X128 || bs == BLOCK_64X128) pcs->mi_grid_base[idx + 16 * pcs->mi_stride]->mbmi.cdef_strength = g;
        if (bs == BLOCK_128X128) pcs->mi_grid_base[idx + 16 * pcs->mi_stride + 16]->mbmi.cdef_strength = g;
    }
    c->cdef_searched = 1;
    free(mask), free(fbb), free(fbs), free(skip);
}

typedef void (*CdefFrameFn)(SequenceControlSet *, PictureControlSet *);
#undef KIND
#define KIND K_CDEF_APPLY
void svt_av1_cdef_frame(SequenceControlSet *scs, PictureControlSet *pcs) {
    static CdefFrameFn orig;
    if (!orig) orig = (CdefFrameFn)dlsym(RTLD_NEXT, "svt_av1_cdef_frame");
    Ctx *c = stage_on(2) && frame_supported(pcs) ? ctx_of(pcs) : NULL;
    if (!c || !c->cdef_searched) {
        if (g_on) count(1);
        return orig(scs, pcs);
    }
    count(0);
    const FrameHeader *fh = &pcs->ppcs->frm_hdr;
    SvtGpuCdefParams   prm;
    memset(&prm, 0, sizeof prm);
    prm.cdef_damping = (uint8_t)fh->cdef_params.cdef_damping;
    prm.cdef_bits    = (uint8_t)fh->cdef_params.cdef_bits;
    for (int j = 0; j < (1 << prm.cdef_bits); j++)
        prm.cdef_y_strength[j] = (uint8_t)fh->cdef_params.cdef_y_strength[j],
        prm.cdef_uv_strength[j] = (uint8_t)fh->cdef_params.cdef_uv_strength[j];
    GPU(svtgpu_cdef_apply_frame(c->cdef, c->D, c->O, &prm, NULL));
    EbPictureBufferDesc *recon;
    svt_aom_get_recon_pic(pcs, &recon, scs->is_16bit_pipeline);
    download_pic(c->O, recon, scs->is_16bit_pipeline, 0, 3);
    c->cdef_searched = 0;
}

/* ========================== loop restoration ========================== */
static int lr_supported(PictureControlSet *pcs) {
    Av1Common *cm = pcs->ppcs->av1_cm;
    if (!frame_supported(pcs)) return 0;
    if (cm->wn_filter_ctrls.enabled && cm->wn_filter_ctrls.use_prev_frame_coeffs) return 0;
    if (cm->sg_filter_ctrls.enabled && cm->sg_filter_ctrls.step_range < 16) return 0; /* reference-based ep range */
    return !cm->use_boundaries_in_rest_search; /* the device search runs without stripe boundaries */
}
static void lr_controls(PictureControlSet *pcs, SvtGpuLrSearchControls *lc) {
    Av1Common        *cm = pcs->ppcs->av1_cm;
    const Macroblock *x  = pcs->ppcs->av1x;
    memset(lc, 0, sizeof *lc);
    lc->wn_enabled                 = cm->wn_filter_ctrls.enabled;
    lc->wn_use_chroma              = cm->wn_filter_ctrls.use_chroma;
    lc->wn_filter_tap_lvl          = cm->wn_filter_ctrls.filter_tap_lvl;
    lc->wn_use_refinement          = cm->wn_filter_ctrls.use_refinement;
    lc->wn_max_one_refinement_step = cm->wn_filter_ctrls.max_one_refinement_step;
    lc->sg_enabled                 = cm->sg_filter_ctrls.enabled;
    lc->sg_use_chroma              = cm->sg_filter_ctrls.use_chroma;
    for (int k = 0; k < 2; k++) {
        lc->sg_start_ep[k] = cm->sg_filter_ctrls.start_ep[k], lc->sg_end_ep[k] = cm->sg_filter_ctrls.end_ep[k];
        lc->sg_ep_inc[k] = cm->sg_filter_ctrls.ep_inc[k], lc->sg_refine[k] = cm->sg_filter_ctrls.refine[k];
    }
    lc->rdmult = x->rdmult;
    for (int k = 0; k < 3; k++) lc->switchable_restore_cost[k] = x->switchable_restore_cost[k];
    for (int k = 0; k < 2; k++) lc->wiener_restore_cost[k] = x->wiener_restore_cost[k];
    for (int k = 0; k < 2; k++) lc->sgrproj_restore_cost[k] = x->sgrproj_restore_cost[k];
}

typedef void (*SegSearchFn)(int32_t *, Yv12BufferConfig *, const Yv12BufferConfig *, Yv12BufferConfig *,
                            PictureControlSet *, uint32_t);
void restoration_seg_search(int32_t *rst_tmpbuf, Yv12BufferConfig *org_fts, const Yv12BufferConfig *src,
                            Yv12BufferConfig *trial_frame_rst, PictureControlSet *pcs, uint32_t segment_index) {
    static SegSearchFn orig;
    if (!orig) orig = (SegSearchFn)dlsym(RTLD_NEXT, "restoration_seg_search");
    if (stage_on(4) && lr_supported(pcs)) {
        /* the device searches the whole frame in rest_finish_search; the one side effect the reference search has on
         * the encoder's picture is kept: it extends the CDEF output's borders in place from the crop size
         * (EbRestorationPick.c:1497-1519), which for a picture off the 8-sample grid rewrites the columns / rows
         * between the crop and the padded size that the reference picture keeps */
        Av1Common *cm  = pcs->ppcs->av1_cm;
        const int  pe  = ((cm->wn_filter_ctrls.enabled && cm->wn_filter_ctrls.use_chroma) ||
                        (cm->sg_filter_ctrls.enabled && cm->sg_filter_ctrls.use_chroma)) ? 2 : 0;
        svt_block_on_mutex(pcs->rest_search_mutex);
        for (int plane = 0; plane <= pe; plane++) {
            if (pcs->rest_extend_flag[plane]) continue;
            const int is_uv = plane > 0, pw = org_fts->crop_widths[is_uv], ph = org_fts->crop_heights[is_uv];
            const int pad16 = (pw % 16) ? 16 - (pw % 16) : 0;
            svt_extend_frame(org_fts->buffers[plane], pw, ph, org_fts->strides[is_uv], RESTORATION_BORDER + 1 + pad16,
                             RESTORATION_BORDER, cm->use_highbitdepth);
            pcs->rest_extend_flag[plane] = TRUE;
        }
        svt_release_mutex(pcs->rest_search_mutex);
        return;
    }
    orig(rst_tmpbuf, org_fts, src, trial_frame_rst, pcs, segment_index);
}

#undef KIND
#define KIND K_LR_SEARCH
void rest_finish_search(PictureControlSet *pcs) {
    static FinishFn orig;
    if (!orig) orig = (FinishFn)dlsym(RTLD_NEXT, "rest_finish_search");
    if (!stage_on(4) || !lr_supported(pcs)) {
        if (stage_on(4)) count(1);
        return orig(pcs);
    }
    count(0);
    SequenceControlSet *scs  = pcs->scs;
    Av1Common          *cm   = pcs->ppcs->av1_cm;
    Ctx                *c    = ctx_of(pcs);
    const int           is16 = scs->is_16bit_pipeline;
    int32_t             us[3];
    for (int p = 0; p < 3; p++) us[p] = pcs->rst_info[p].restoration_unit_size;
    if (!c->lr || memcmp(us, c->lr_units, sizeof us)) {
        if (c->lr) svtgpu_lr_state_destroy(c->lr);
        GPU(svtgpu_lr_state_create(g_ctx, c->cw, c->ch, us, &c->lr)); /* the crop size */
        memcpy(c->lr_units, us, sizeof us);
    }
    /* the CDEF output the search reads (EbRestProcess.c:562) and the source (:563) */
    EbPictureBufferDesc *recon;
    svt_aom_get_recon_pic(pcs, &recon, is16);
    upload_pic(c->O, recon, is16, 0, 3);
    upload_pic(c->S, is16 ? pcs->input_frame16bit : pcs->ppcs->enhanced_unscaled_pic, is16, 0, 3);
    SvtGpuLrSearchControls lc;
    lr_controls(pcs, &lc);
    SvtGpuLrUnitSearch *rec[3];
    int32_t             n[3];
    for (int p = 0; p < 3; p++) {
        int32_t hu, vu;
        GPU(svtgpu_lr_units(c->lr, p, &hu, &vu));
        n[p]   = hu * vu;
        rec[p] = calloc((size_t)n[p], sizeof **rec);
    }
    int32_t ft[3];
    GPU(svtgpu_lr_search_frame(c->lr, c->O, c->S, &lc, ft, rec, NULL));
    const int nplanes = ((lc.wn_enabled && lc.wn_use_chroma) || (lc.sg_enabled && lc.sg_use_chroma)) ? 3 : 1;
    /* the units for the encoder's rst_info: the whole frame's host finish over the records (its RestUnitSearchInfo
     * shared by the planes, as rest_finish_search's: a chroma plane's switchable pass reads luma's entries for a type
     * chroma does not search -- presets 3-9 with Wiener level 5), which must agree with the device finish's types */
    SvtGpuRestUnit *units[3];
    int32_t         t[3];
    for (int p = 0; p < 3; p++) units[p] = calloc((size_t)n[p], sizeof **units);
    GPU(svtgpu_lr_finish_frame(&lc, n, (const SvtGpuLrUnitSearch *const *)rec, t, units));
    for (int p = 0; p < 3; p++) {
        RestorationInfo *ri = &pcs->rst_info[p];
        if (p >= nplanes) { /* luma-only search: chroma off (EbRestorationPick.c:1626-1629) */
            ri->frame_restoration_type = RESTORE_NONE;
            free(units[p]);
            continue;
        }
        if (t[p] != ft[p]) die("lr finish: the host finish's frame type differs from the device's", t[p]);
        ri->frame_restoration_type = (RestorationType)t[p];
        if (t[p] != RESTORE_NONE)
            for (int u = 0; u < n[p]; u++) { /* copy_unit_info (EbRestorationPick.c:1202-1209) */
                RestorationUnitInfo  *ui = &ri->unit_info[u];
                const SvtGpuRestUnit *g  = &units[p][u];
                ui->restoration_type     = (RestorationType)g->type;
                if (g->type == RESTORE_WIENER)
                    for (int k = 0; k < 8; k++) ui->wiener_info.vfilter[k] = g->vfilter[k], ui->wiener_info.hfilter[k] = g->hfilter[k];
                else if (g->type == RESTORE_SGRPROJ)
                    ui->sgrproj_info.ep = g->ep, ui->sgrproj_info.xqd[0] = g->xqd[0], ui->sgrproj_info.xqd[1] = g->xqd[1];
            }
        /* the device finish's units (svtgpu_lr_read_units) must be the same picks */
        SvtGpuRestUnit *dev = calloc((size_t)n[p], sizeof *dev);
        GPU(svtgpu_lr_read_units(c->lr, p, dev, NULL));
        for (int u = 0; u < n[p] && t[p] != RESTORE_NONE; u++)
            if (dev[u].type != units[p][u].type || (dev[u].type == RESTORE_WIENER && memcmp(dev[u].vfilter, units[p][u].vfilter, 32)) ||
                (dev[u].type == RESTORE_SGRPROJ && (dev[u].ep != units[p][u].ep || dev[u].xqd[0] != units[p][u].xqd[0] ||
                                                    dev[u].xqd[1] != units[p][u].xqd[1])))
                die("lr finish: the device finish's unit differs from the host finish's", u);
        free(dev);
        /* search_sgrproj_seg counts each unit's best ep (EbRestorationPick.c:1256; the frame's ep for later frames) */
        if (lc.sg_enabled && (p == 0 || lc.sg_use_chroma))
            for (int u = 0; u < n[p]; u++) cm->sg_frame_ep_cnt[rec[p][u].sgrproj.ep]++;
        free(units[p]);
    }
    for (int p = 0; p < 3; p++) c->lr_ft[p] = pcs->rst_info[p].frame_restoration_type, free(rec[p]);
    if (c->lr_ft[0] || c->lr_ft[1] || c->lr_ft[2]) count_kind(0, K_LR_ON), g_calls--;
    c->lr_searched = 1;
}

typedef void (*LrFrameFn)(int32_t *, Yv12BufferConfig *, Av1Common *, int32_t);
#undef KIND
#define KIND K_LR_APPLY
void svt_av1_loop_restoration_filter_frame(int32_t *rst_tmpbuf, Yv12BufferConfig *frame, Av1Common *cm,
                                           int32_t optimized_lr) {
    static LrFrameFn orig;
    if (!orig) orig = (LrFrameFn)dlsym(RTLD_NEXT, "svt_av1_loop_restoration_filter_frame");
    PictureControlSet *pcs = cm->child_pcs;
    Ctx               *c   = stage_on(4) && frame_supported(pcs) ? ctx_of(pcs) : NULL;
    if (!c || !c->lr_searched) {
        if (g_on) count(1);
        return orig(rst_tmpbuf, frame, cm, optimized_lr);
    }
    if (!c->d_valid) { /* no deblocked copy of this picture: the encoder's own apply (its boundary buffers) */
        count(1);
        c->lr_searched = 0;
        return orig(rst_tmpbuf, frame, cm, optimized_lr);
    }
    count(0);
    void   *pl[3];
    int32_t st[3];
    yv12_planes(frame, cm->use_highbitdepth, pl, st);
    for (int q = 0; q < 3; q++) GPU(svtgpu_frame_upload(c->O, q, pl[q], st[q], NULL));
    GPU(svtgpu_lr_apply_frame(c->lr, c->D, c->O, c->L, c->lr_ft, NULL));
    for (int q = 0; q < 3; q++) GPU(svtgpu_frame_download(c->L, q, pl[q], st[q], NULL));
    GPU(svtgpu_synchronize(g_ctx, NULL));
    c->lr_searched = 0, c->d_valid = 0;
}

/* ============================== CCSO (the ccso build only) ============================== */
/* the process body passes host buffers: ext_rec_y ((H + 10) x (W + 10)) and the planes' org / rec (H x W each, the
 * luma width as stride) of the unpadded size W x H (svt_av1_setup_dst_planes, EbDeblockingFilter.c:95-137) */
static int ccso_supported(PictureControlSet *pcs) {
    return frame_supported(pcs) && !pcs->scs->is_16bit_pipeline && pcs->scs->static_config.encoder_bit_depth == 8 &&
           !pcs->scs->seq_header.color_config.mono_chrome;
}
static void ccso_dims(PictureControlSet *pcs, int *W, int *H) {
    SequenceControlSet *scs = pcs->scs;
    *W = scs->max_input_luma_width - scs->max_input_pad_right, *H = scs->max_input_luma_height - scs->max_input_pad_bottom;
}
static void ccso_buffers(Ctx *c, int W, int H) {
    if (c->ccso) return;
    GPU(svtgpu_ccso_state_create(g_ctx, W, H, &c->ccso));
    GPU(svtgpu_buffer_alloc(g_ctx, sizeof(uint16_t) * (size_t)(W + 10) * (H + 10), &c->d_ext));
    for (int p = 0; p < 3; p++) {
        GPU(svtgpu_buffer_alloc(g_ctx, sizeof(uint16_t) * (size_t)W * H, &c->d_org[p]));
        GPU(svtgpu_buffer_alloc(g_ctx, sizeof(uint16_t) * (size_t)W * H, &c->d_rec[p]));
    }
}
/* the block flags of one plane in the mode-info grid: mbmi.ccso_blk_{y,u,v} at (64 y, 64 x) (EbPickccso.c:731-751) */
static uint8_t *ccso_flag(PictureControlSet *pcs, int plane, int y, int x, uint8_t *v) {
    MbModeInfo *m = &pcs->mi_grid_base[64 * y * pcs->mi_stride + 64 * x]->mbmi;
    if (v) {
        if (plane == 0) m->ccso_blk_y = *v;
        else if (plane == 1) m->ccso_blk_u = *v;
        else m->ccso_blk_v = *v;
        return v;
    }
    static __thread uint8_t r;
    r = plane == 0 ? m->ccso_blk_y : plane == 1 ? m->ccso_blk_u : m->ccso_blk_v;
    return &r;
}

typedef void (*CcsoSearchFn)(PictureControlSet *, MacroblockdPlane *, int, const uint16_t *, uint16_t *[3],
                             uint16_t *[3]);
#undef KIND
#define KIND K_CCSO_SEARCH
void ccso_search(PictureControlSet *pcs, MacroblockdPlane *pd, int rdmult, const uint16_t *ext_rec_y,
                 uint16_t *rec_uv[3], uint16_t *org_uv[3]) {
    static CcsoSearchFn orig;
    if (!orig) orig = (CcsoSearchFn)dlsym(RTLD_NEXT, "ccso_search");
    if (!stage_on(8) || !ccso_supported(pcs)) {
        if (g_on) count(1);
        return orig(pcs, pd, rdmult, ext_rec_y, rec_uv, org_uv);
    }
    Ctx *c = ctx_of(pcs);
    int  W, H;
    ccso_dims(pcs, &W, &H);
    ccso_buffers(c, W, H);
    GPU(svtgpu_buffer_upload(c->d_ext, ext_rec_y, sizeof(uint16_t) * (size_t)(W + 10) * (H + 10), NULL));
    for (int p = 0; p < 3; p++) {
        GPU(svtgpu_buffer_upload(c->d_org[p], org_uv[p], sizeof(uint16_t) * (size_t)W * H, NULL));
        GPU(svtgpu_buffer_upload(c->d_rec[p], rec_uv[p], sizeof(uint16_t) * (size_t)W * H, NULL));
    }
    const uint16_t *org[3] = {c->d_org[0], c->d_org[1], c->d_org[2]}, *rec[3] = {c->d_rec[0], c->d_rec[1], c->d_rec[2]};
    SvtGpuCcsoParams prm[3];
    uint8_t         *flags[3];
    int32_t          nv[3], nh[3], ff = 0;
    for (int p = 0; p < 3; p++) {
        GPU(svtgpu_ccso_grid(W, H, p, &nv[p], &nh[p]));
        flags[p] = malloc((size_t)nv[p] * nh[p]);
    }
    FrameHeader *fh = &pcs->ppcs->frm_hdr;
    const int    rc = svtgpu_ccso_search_frame(c->ccso, c->d_ext, org, rec, 8, rdmult,
                                               fh->quantization_params.base_q_idx, prm, flags, &ff, NULL);
    if (rc != 1) { /* 1: the weighted rdmult overflows and the reference returns before searching (EbPickccso.c:790) */
        GPU(rc);
        for (int p = 0; p < 3; p++) { /* the header fields and grid flags derive_ccso_filter writes (:725-757) */
            fh->ccso_info.ccso_enable[p] = prm[p].enable;
            if (!prm[p].enable) continue;
            for (int y = 0; y < nv[p]; y++)
                for (int x = 0; x < nh[p]; x++) ccso_flag(pcs, p, y, x, &flags[p][y * nh[p] + x]);
            memcpy(fh->ccso_info.filter_offset[p], prm[p].filter_offset, sizeof prm[p].filter_offset);
            fh->ccso_info.quant_idx[p]          = prm[p].quant_idx;
            fh->ccso_info.ext_filter_support[p] = prm[p].ext_filter_support;
            fh->ccso_info.ccso_bo_only[p]       = prm[p].bo_only;
            fh->ccso_info.max_band_log2[p]      = prm[p].max_band_log2;
            fh->ccso_info.edge_clf[p]           = prm[p].edge_clf;
            pthread_mutex_lock(&g_mu), g_kind[K_CCSO_ON]++, pthread_mutex_unlock(&g_mu);
        }
        fh->ccso_info.ccso_frame_flag = ff != 0; /* CONFIG_D143_CCSO_FM_FLAG (:804-813) */
    }
    for (int p = 0; p < 3; p++) free(flags[p]);
    count(0);
}

typedef void (*CcsoFrameFn)(EbPictureBufferDesc *, PictureControlSet *, MacroblockdPlane *, uint16_t *);
#undef KIND
#define KIND K_CCSO_APPLY
void ccso_frame(EbPictureBufferDesc *frame, PictureControlSet *pcs, MacroblockdPlane *pd, uint16_t *ext_rec_y) {
    static CcsoFrameFn orig;
    if (!orig) orig = (CcsoFrameFn)dlsym(RTLD_NEXT, "ccso_frame");
    if (!stage_on(8) || !ccso_supported(pcs) || frame->bit_depth != EB_EIGHT_BIT) {
        if (g_on) count(1);
        return orig(frame, pcs, pd, ext_rec_y);
    }
    Ctx *c = ctx_of(pcs);
    int  W, H;
    ccso_dims(pcs, &W, &H);
    ccso_buffers(c, W, H);
    GPU(svtgpu_buffer_upload(c->d_ext, ext_rec_y, sizeof(uint16_t) * (size_t)(W + 10) * (H + 10), NULL));
    const FrameHeader *fh = &pcs->ppcs->frm_hdr;
    for (int p = 0; p < 3; p++) {
        if (!fh->ccso_info.ccso_enable[p]) continue;
        /* the plane as svt_av1_setup_dst_planes1 points at it (EbCcso.c:121-183, 8-bit buffers) */
        const int st = p == 0 ? frame->stride_y : p == 1 ? frame->stride_cb : frame->stride_cr;
        uint8_t  *b  = p == 0 ? frame->buffer_y + frame->org_x + frame->org_y * frame->stride_y
                     : (p == 1 ? frame->buffer_cb : frame->buffer_cr) + (frame->org_x + frame->org_y * st) / 2;
        const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H;
        const size_t n = (size_t)(ph - 1) * st + pw;
        if (!c->d_pl[p] || c->pl_bytes[p] < n) {
            if (c->d_pl[p]) svtgpu_buffer_free(c->d_pl[p]);
            GPU(svtgpu_buffer_alloc(g_ctx, n, &c->d_pl[p]));
            c->pl_bytes[p] = n;
        }
        SvtGpuCcsoParams prm;
        memset(&prm, 0, sizeof prm);
        prm.enable = 1, prm.bo_only = fh->ccso_info.ccso_bo_only[p], prm.quant_idx = fh->ccso_info.quant_idx[p];
        prm.ext_filter_support = fh->ccso_info.ext_filter_support[p];
        prm.max_band_log2 = (uint8_t)fh->ccso_info.max_band_log2[p], prm.edge_clf = fh->ccso_info.edge_clf[p];
        memcpy(prm.filter_offset, fh->ccso_info.filter_offset[p], sizeof prm.filter_offset);
        int32_t nv, nh;
        GPU(svtgpu_ccso_grid(W, H, p, &nv, &nh));
        uint8_t *flags = malloc((size_t)nv * nh);
        for (int y = 0; y < nv; y++)
            for (int x = 0; x < nh; x++) flags[y * nh + x] = *ccso_flag(pcs, p, y, x, NULL);
        GPU(svtgpu_buffer_upload(c->d_pl[p], b, n, NULL));
        GPU(svtgpu_ccso_apply_plane(c->ccso, c->d_ext, p, 8, c->d_pl[p], 8, st, &prm, flags, NULL));
        GPU(svtgpu_buffer_download(b, c->d_pl[p], n, NULL));
        free(flags);
    }
    count(0);
}
