/*
 * gen_golden_pipe.c — whole-frame pipeline golden vectors (test infrastructure; never shipped).
 *
 * Runs the REFERENCE's own frame-level code, compiled from /root/reference by oracle/ref.mk, in the order the
 * encoder's DLF -> CDEF -> REST processes run it (EbDlfProcess.c:96-136, EbCdefProcess.c:398-520 / :663-670,
 * EbRestProcess.c:552-630), on a recon/source pair and a mode-info grid handed in by tests/golden/
 * make_pipeline_golden.py:
 *   svt_av1_loop_filter_init + svt_av1_pick_filter_level(FULL_IMAGE) + svt_av1_loop_filter_frame, or at the SB-based
 *   DLF levels (3-5) the encode loop's pick_filter_level(FROM_Q) + svt_aom_loop_filter_sb per SB in raster order
 *   svt_aom_link_eb_to_aom_buffer_desc + svt_av1_loop_restoration_save_boundary_lines(after_cdef = 0)
 *   cdef_seg_search (per segment) + finish_cdef_search + svt_av1_cdef_frame
 *   svt_av1_loop_restoration_save_boundary_lines(after_cdef = 1)
 *   restoration_seg_search (per segment) + rest_finish_search + svt_av1_loop_restoration_filter_frame
 * with every kernel bound to its C version.  The controls come from the reference's own level tables
 * (EncModeConfig.c, through ref_mode_config.c) and the CDEF lambda from its own lambda assignment.
 *
 *   gen_golden_pipe pipe  <in.bin> <out.bin>   one frame (input layout: tests/pipeline_cases.py write_input)
 *   gen_golden_pipe byq   <out.bin>            svt_av1_pick_filter_level(LPF_PICK_FROM_Q) and qp_based_dlf_param
 *   gen_golden_pipe ctrls <out.bin>            the CDEF / DLF / Wiener / self-guided control tables of every level
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbPictureControlSet.h"
#include "EbSequenceControlSet.h"
#include "EbDeblockingFilter.h"
#include "EbRestoration.h"
#include "EbReferenceObject.h"
#include "Av1Common.h"
#include "common_dsp_rtcd.h"
#include "aom_dsp_rtcd.h"
#include "EbCodingUnit.h"
#include "EbThreads.h"
#include "golden_io.h"

void        svt_av1_loop_filter_init(PictureControlSet *pcs);
void        svt_aom_loop_filter_sb(EbPictureBufferDesc *frame_buffer, PictureControlSet *pcs, int32_t mi_row,
                                   int32_t mi_col, int32_t plane_start, int32_t plane_end, uint8_t last_col);
void        svt_av1_loop_filter_frame_init(FrameHeader *frm_hdr, LoopFilterInfoN *lf_info, int32_t plane_start,
                                           int32_t plane_end);
void        svt_av1_loop_filter_frame(EbPictureBufferDesc *frame_buffer, PictureControlSet *pcs, int32_t plane_start,
                                      int32_t plane_end);
EbErrorType qp_based_dlf_param(PictureControlSet *pcs, int32_t *filter_level_y, int32_t *filter_level_uv);
void        finish_cdef_search(PictureControlSet *pcs);
void        svt_av1_cdef_frame(SequenceControlSet *scs, PictureControlSet *pcs);
void        svt_av1_loop_restoration_filter_frame(int32_t *rst_tmpbuf, Yv12BufferConfig *frame, Av1Common *cm,
                                                  int32_t optimized_lr);
void        svt_av1_loop_restoration_save_boundary_lines(const Yv12BufferConfig *frame, Av1Common *cm, int32_t after_cdef);
EbErrorType svt_av1_alloc_restoration_buffers(PictureControlSet *pcs, Av1Common *cm);
void        restoration_seg_search(int32_t *rst_tmpbuf, Yv12BufferConfig *org_fts, const Yv12BufferConfig *src,
                                   Yv12BufferConfig *trial_frame_rst, PictureControlSet *pcs, uint32_t segment_index);
void        rest_finish_search(PictureControlSet *pcs);
/* harness units compiled with the reference's own EbCdefProcess.c / EncModeConfig.c */
void ref_cdef_seg_search(PictureControlSet *pcs, SequenceControlSet *scs, uint32_t segment_index);
void ref_set_cdef_controls(PictureParentControlSet *pcs, uint8_t cdef_level, int fast_decode);
void ref_set_wn_filter_ctrls(Av1Common *cm, uint8_t lvl);
void ref_set_sg_filter_ctrls(Av1Common *cm, uint8_t lvl);
void ref_set_dlf_controls(PictureParentControlSet *pcs, uint8_t lvl);

static void bind_c_kernels(void) {
    svt_aom_lpf_horizontal_4               = svt_aom_lpf_horizontal_4_c;
    svt_aom_lpf_horizontal_6               = svt_aom_lpf_horizontal_6_c;
    svt_aom_lpf_horizontal_8               = svt_aom_lpf_horizontal_8_c;
    svt_aom_lpf_horizontal_14              = svt_aom_lpf_horizontal_14_c;
    svt_aom_lpf_vertical_4                 = svt_aom_lpf_vertical_4_c;
    svt_aom_lpf_vertical_6                 = svt_aom_lpf_vertical_6_c;
    svt_aom_lpf_vertical_8                 = svt_aom_lpf_vertical_8_c;
    svt_aom_lpf_vertical_14                = svt_aom_lpf_vertical_14_c;
    svt_aom_highbd_lpf_horizontal_4        = svt_aom_highbd_lpf_horizontal_4_c;
    svt_aom_highbd_lpf_horizontal_6        = svt_aom_highbd_lpf_horizontal_6_c;
    svt_aom_highbd_lpf_horizontal_8        = svt_aom_highbd_lpf_horizontal_8_c;
    svt_aom_highbd_lpf_horizontal_14       = svt_aom_highbd_lpf_horizontal_14_c;
    svt_aom_highbd_lpf_vertical_4          = svt_aom_highbd_lpf_vertical_4_c;
    svt_aom_highbd_lpf_vertical_6          = svt_aom_highbd_lpf_vertical_6_c;
    svt_aom_highbd_lpf_vertical_8          = svt_aom_highbd_lpf_vertical_8_c;
    svt_aom_highbd_lpf_vertical_14         = svt_aom_highbd_lpf_vertical_14_c;
    svt_log2f                              = svt_aom_log2f_32;
    svt_spatial_full_distortion_kernel     = svt_spatial_full_distortion_kernel_c;
    svt_full_distortion_kernel16_bits      = svt_full_distortion_kernel16_bits_c;
    svt_cdef_filter_block                  = svt_cdef_filter_block_c;
    svt_aom_cdef_find_dir                  = svt_aom_cdef_find_dir_c;
    svt_aom_cdef_find_dir_dual             = svt_aom_cdef_find_dir_dual_c;
    svt_compute_cdef_dist_16bit            = svt_aom_compute_cdef_dist_c;
    svt_compute_cdef_dist_8bit             = svt_aom_compute_cdef_dist_8bit_c;
    svt_search_one_dual                    = svt_search_one_dual_c;
    svt_aom_copy_rect8_8bit_to_16bit       = svt_aom_copy_rect8_8bit_to_16bit_c;
    svt_av1_wiener_convolve_add_src        = svt_av1_wiener_convolve_add_src_c;
    svt_av1_highbd_wiener_convolve_add_src = svt_av1_highbd_wiener_convolve_add_src_c;
    svt_av1_selfguided_restoration         = svt_av1_selfguided_restoration_c;
    svt_apply_selfguided_restoration       = svt_apply_selfguided_restoration_c;
    svt_memcpy                             = svt_memcpy_c;
    svt_av1_compute_stats                  = svt_av1_compute_stats_c;
    svt_av1_compute_stats_highbd           = svt_av1_compute_stats_highbd_c;
    svt_get_proj_subspace                  = svt_get_proj_subspace_c;
    svt_av1_lowbd_pixel_proj_error         = svt_av1_lowbd_pixel_proj_error_c;
    svt_av1_highbd_pixel_proj_error        = svt_av1_highbd_pixel_proj_error_c;
    svt_aom_mse16x16                       = svt_aom_mse16x16_c;
    svt_aom_highbd_8_mse16x16              = svt_aom_highbd_8_mse16x16_c;
}

#ifdef SVTGPU_BIND
/* rtcd_pipe: the same frame code with every RTCD pointer bound to libsvtgpu's device shims by the encoder's own install
 * header (include/svtgpu_rtcd.h): each assignment compiles under -Werror=incompatible-pointer-types
 * without a cast */
#include "EbMcp.h"
#include "svtgpu_rtcd.h"
static void bind_device_kernels(void) {
    svtgpu_install_filter_rtcd();
    svtgpu_install_me_md_rtcd(); /* compiled and installed; the frame code here calls none of them */
    svtgpu_install_ccso_rtcd();  /* likewise (CCSO is dead in this encoder) */
}
/* the frame-buffer functions the reference calls directly (not through RTCD): a pointer of each one's type */
void bind_check_frame(void);
void bind_check_frame(void) {
    __typeof__(&svt_aom_generate_padding)       pad8  = svtgpu_aom_generate_padding;
    __typeof__(&svt_aom_generate_padding16_bit) pad16 = svtgpu_aom_generate_padding16_bit;
    __typeof__(&svt_extend_frame)               ext   = svtgpu_extend_frame;
    (void)pad8, (void)pad16, (void)ext;
}
#endif

/* input header (int32), written by tests/pipeline_cases.py:write_input */
enum {
    I_MAGIC, I_W, I_H, I_BD, I_Q, I_CDEF_LVL, I_DLF_LVL, I_WN_LVL, I_SG_LVL, I_LF0, I_LF1, I_LFU, I_LFV, I_SHARP,
    I_MRD, I_TL, I_FRAME_TYPE, I_UPDATE_TYPE, I_HIER, I_RDMULT, I_SW0, I_SW1, I_SW2, I_WC0, I_WC1, I_SC0, I_SC1,
    I_US_Y, I_US_UV, I_CDEF_SC, I_CDEF_SR, I_REST_SC, I_REST_SR, I_ONLY4X4, I_SB, I_PRED_Y, I_PRED_UV, I_MESAD,
    I_IN_RES, I_SLICE_TYPE, I_COUNT = 64
};
#define PIPE_MAGIC 0x45504950

static EbErrorType new_pic(EbPictureBufferDesc **out, int w, int h, int hbd, int pad) {
    EbPictureBufferDescInitData d;
    memset(&d, 0, sizeof d);
    d.max_width          = (uint16_t)w;
    d.max_height         = (uint16_t)h;
    d.bit_depth          = hbd ? EB_TEN_BIT : EB_EIGHT_BIT;
    d.color_format       = EB_YUV420;
    d.buffer_enable_mask = PICTURE_BUFFER_DESC_FULL_MASK;
    d.left_padding = d.right_padding = d.top_padding = d.bot_padding = (uint16_t)pad;
    EbPictureBufferDesc *p;
    EB_NEW(p, svt_recon_picture_buffer_desc_ctor, (EbPtr)&d);
    *out = p;
    return EB_ErrorNone;
}

static void *plane_ptr(EbPictureBufferDesc *p, int pl, int *stride) {
    const int hbd = p->bit_depth > EB_EIGHT_BIT;
    const int st  = pl == 0 ? p->stride_y : pl == 1 ? p->stride_cb : p->stride_cr;
    uint8_t  *b   = pl == 0 ? p->buffer_y : pl == 1 ? p->buffer_cb : p->buffer_cr;
    const int ox = pl ? p->org_x / 2 : p->org_x, oy = pl ? p->org_y / 2 : p->org_y;
    *stride = st;
    return b + ((size_t)(oy * st + ox) << hbd);
}

static void put_pic(EbPictureBufferDesc *p, int pl, const uint16_t *src, int w, int h) {
    int   st;
    void *b = plane_ptr(p, pl, &st);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            if (p->bit_depth > EB_EIGHT_BIT)
                ((uint16_t *)b)[(size_t)y * st + x] = src[(size_t)y * w + x];
            else
                ((uint8_t *)b)[(size_t)y * st + x] = (uint8_t)src[(size_t)y * w + x];
        }
}

static void emit_pic(GoldenFile *g, const char *tag, EbPictureBufferDesc *p, int W, int H) {
    for (int pl = 0; pl < 3; pl++) {
        const int w = pl ? W / 2 : W, h = pl ? H / 2 : H;
        int       st;
        void     *b = plane_ptr(p, pl, &st);
        uint16_t *a = malloc(sizeof(uint16_t) * (size_t)w * h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++)
                a[(size_t)y * w + x] = p->bit_depth > EB_EIGHT_BIT ? ((uint16_t *)b)[(size_t)y * st + x]
                                                                   : ((uint8_t *)b)[(size_t)y * st + x];
        char nm[32];
        snprintf(nm, sizeof nm, "%s%d", tag, pl);
        golden_put2(g, nm, 'H', (uint32_t)h, (uint32_t)w, a);
        free(a);
    }
}

static void *read_all(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        exit(1);
    }
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void *b = malloc(*n);
    if (fread(b, 1, *n, f) != *n) {
        fprintf(stderr, "short read %s\n", path);
        exit(1);
    }
    fclose(f);
    return b;
}

/* the Wiener statistics of every searched unit, recorded from the reference's own svt_av1_compute_stats(_highbd)_c
 * calls inside restoration_seg_search: {plane, win, h_start, h_end, v_start, v_end} and M / H per call */
static struct {
    EbPictureBufferDesc *pic;
    int                  n, cap_m, cap_h, nm, nh;
    int32_t             *meta;
    int64_t             *M, *H;
} g_rec;
static void rec_stats(int32_t win, const uint8_t *dgd, int32_t hs, int32_t he, int32_t vs, int32_t ve, const int64_t *M,
                      const int64_t *H) {
    const int win2 = win * win, hbd = g_rec.pic->bit_depth > EB_EIGHT_BIT;
    int       plane = -1;
    for (int p = 0; p < 3; p++) {
        int            st;
        const uint8_t *b  = plane_ptr(g_rec.pic, p, &st);
        const size_t   sz = (size_t)st * (p ? g_rec.pic->height / 2 : g_rec.pic->height) << hbd;
        const uint8_t *a  = hbd ? (const uint8_t *)((uintptr_t)dgd << 1) : dgd;
        if (a >= b && a < b + sz) plane = p;
    }
    g_rec.meta = realloc(g_rec.meta, sizeof(int32_t) * 6 * (g_rec.n + 1));
    int32_t *m = g_rec.meta + 6 * g_rec.n++;
    m[0] = plane, m[1] = win, m[2] = hs, m[3] = he, m[4] = vs, m[5] = ve;
    g_rec.M = realloc(g_rec.M, sizeof(int64_t) * (g_rec.nm + win2));
    g_rec.H = realloc(g_rec.H, sizeof(int64_t) * (g_rec.nh + win2 * win2));
    memcpy(g_rec.M + g_rec.nm, M, sizeof(int64_t) * win2), g_rec.nm += win2;
    memcpy(g_rec.H + g_rec.nh, H, sizeof(int64_t) * win2 * win2), g_rec.nh += win2 * win2;
}
static void rec_compute_stats(int32_t win, const uint8_t *dgd, const uint8_t *src, int32_t hs, int32_t he, int32_t vs,
                              int32_t ve, int32_t ds, int32_t ss, int64_t *M, int64_t *H) {
    svt_av1_compute_stats_c(win, dgd, src, hs, he, vs, ve, ds, ss, M, H);
    rec_stats(win, dgd, hs, he, vs, ve, M, H);
}
static void rec_compute_stats_highbd(int32_t win, const uint8_t *dgd, const uint8_t *src, int32_t hs, int32_t he,
                                     int32_t vs, int32_t ve, int32_t ds, int32_t ss, int64_t *M, int64_t *H,
                                     EbBitDepth bd) {
    svt_av1_compute_stats_highbd_c(win, dgd, src, hs, he, vs, ve, ds, ss, M, H, bd);
    rec_stats(win, dgd, hs, he, vs, ve, M, H);
}

/* ------------------------------------------------------------------------------------------- */
static int run_pipe(const char *in_path, const char *out_path) {
    size_t         nbytes;
    uint8_t       *in  = read_all(in_path, &nbytes);
    const int32_t *hdr = (const int32_t *)in;
    if (hdr[I_MAGIC] != PIPE_MAGIC) {
        fprintf(stderr, "bad input magic\n");
        return 1;
    }
    const int     W = hdr[I_W], H = hdr[I_H], BD = hdr[I_BD], hbd = BD > 8, SB = hdr[I_SB] ? hdr[I_SB] : 64;
    const int     mi_cols = ((W + 7) & ~7) >> 2, mi_rows = ((H + 7) & ~7) >> 2;
    const int8_t *deltas  = (const int8_t *)(hdr + I_COUNT);
    const size_t  ny = (size_t)W * H, nc = ny / 4;
    const uint16_t *src = (const uint16_t *)(deltas + 16);
    const uint16_t *rec = src + ny + 2 * nc;
    const uint8_t  *mi8 = (const uint8_t *)(rec + ny + 2 * nc);
    if ((size_t)((mi8 + (size_t)mi_rows * mi_cols * 8) - in) != nbytes) {
        fprintf(stderr, "input size mismatch\n");
        return 1;
    }

    SequenceControlSet      *scs  = calloc(1, sizeof(*scs));
    PictureParentControlSet *ppcs = calloc(1, sizeof(*ppcs));
    PictureControlSet       *pcs  = calloc(1, sizeof(*pcs));
    Av1Common               *cm   = calloc(1, sizeof(*cm));
    Macroblock              *x    = calloc(1, sizeof(*x));
    EncDecSet               *eds  = calloc(1, sizeof(*eds));
    pcs->scs = ppcs->scs = scs;
    pcs->ppcs            = ppcs;
    ppcs->av1_cm         = cm;
    ppcs->av1x           = x;
    ppcs->enc_dec_ptr    = eds;
    cm->child_pcs        = pcs;
    /* sequence */
    scs->super_block_size                   = (uint8_t)SB;
    scs->sb_size                            = (uint8_t)SB;
    scs->seq_header.sb_size                 = SB == 128 ? BLOCK_128X128 : BLOCK_64X64;
    scs->is_16bit_pipeline                  = (uint8_t)hbd;
    scs->static_config.encoder_bit_depth    = (uint32_t)BD;
    scs->static_config.encoder_color_format = EB_YUV420;
    scs->subsampling_x = scs->subsampling_y = 1;
    scs->max_input_luma_width               = (uint16_t)W;
    scs->max_input_luma_height              = (uint16_t)H;
    scs->seq_header.cdef_level              = (uint8_t)(hdr[I_CDEF_LVL] != 0);
    scs->seq_header.color_config.mono_chrome = 0;
    for (int k = 0; k < SVT_AV1_FRAME_UPDATE_TYPES; k++) scs->static_config.lambda_scale_factors[k] = 128;
    /* picture */
    ppcs->aligned_width = ppcs->render_width = (uint16_t)W;
    ppcs->aligned_height = ppcs->render_height = (uint16_t)H;
    ppcs->enable_restoration                  = 1;
    ppcs->is_ref                              = 0;
    ppcs->temporal_layer_index                = (uint8_t)hdr[I_TL];
    pcs->temporal_layer_index                 = (uint8_t)hdr[I_TL];
    ppcs->hierarchical_levels                 = (uint8_t)hdr[I_HIER];
    ppcs->update_type                         = (SvtAv1FrameUpdateType)hdr[I_UPDATE_TYPE];
    ppcs->pred_structure                      = 2; /* random access; every entry of the table is av1_lambda_assign */
    ppcs->cdef_level                          = (int8_t)hdr[I_CDEF_LVL];
    FrameHeader *fh                           = &ppcs->frm_hdr;
    fh->frame_type                            = (FrameType)hdr[I_FRAME_TYPE];
    fh->quantization_params.base_q_idx        = (uint8_t)hdr[I_Q];
    fh->tx_mode                               = hdr[I_ONLY4X4] ? ONLY_4X4 : TX_MODE_SELECT;
    struct LoopFilter *lf                     = &fh->loop_filter_params;
    lf->filter_level[0]                       = hdr[I_LF0];
    lf->filter_level[1]                       = hdr[I_LF1];
    lf->filter_level_u                        = hdr[I_LFU];
    lf->filter_level_v                        = hdr[I_LFV];
    lf->sharpness_level                       = hdr[I_SHARP];
    lf->mode_ref_delta_enabled                = (uint8_t)hdr[I_MRD];
    for (int k = 0; k < 8; k++) lf->ref_deltas[k] = deltas[k];
    for (int k = 0; k < 2; k++) lf->mode_deltas[k] = deltas[8 + k];
    /* controls from the reference's own level tables */
    ref_set_dlf_controls(ppcs, (uint8_t)hdr[I_DLF_LVL]);
    ref_set_cdef_controls(ppcs, (uint8_t)hdr[I_CDEF_LVL], 0);
    ppcs->cdef_ctrls.pred_y_f  = (int8_t)hdr[I_PRED_Y]; /* the MDC process derives these from the references */
    ppcs->cdef_ctrls.pred_uv_f = (int8_t)hdr[I_PRED_UV];
    ref_set_wn_filter_ctrls(cm, (uint8_t)hdr[I_WN_LVL]);
    ref_set_sg_filter_ctrls(cm, (uint8_t)hdr[I_SG_LVL]);
    /* frame geometry */
    cm->frm_size.frame_width = cm->frm_size.superres_upscaled_width = W;
    cm->frm_size.frame_height = cm->frm_size.superres_upscaled_height = H;
    cm->subsampling_x = cm->subsampling_y = 1;
    cm->use_highbitdepth                  = hbd;
    cm->bit_depth                         = BD;
    cm->mi_rows                           = mi_rows;
    cm->mi_cols                           = mi_cols;
    cm->mi_stride                         = mi_cols;
    /* rate inputs of the restoration search */
    x->rdmult = hdr[I_RDMULT];
    for (int k = 0; k < 3; k++) x->switchable_restore_cost[k] = hdr[I_SW0 + k];
    for (int k = 0; k < 2; k++) x->wiener_restore_cost[k] = hdr[I_WC0 + k];
    for (int k = 0; k < 2; k++) x->sgrproj_restore_cost[k] = hdr[I_SC0 + k];
    /* mode info: one MbModeInfo per 4x4 (the reference duplicates block data per mi, EbEncCdef.c:768) */
    MbModeInfo *cells = calloc((size_t)mi_rows * mi_cols, sizeof(MbModeInfo));
    ModeInfo  **grid  = calloc((size_t)mi_rows * mi_cols, sizeof(ModeInfo *));
    for (int k = 0; k < mi_rows * mi_cols; k++) {
        MbModeInfo *m               = &cells[k];
        const uint8_t *r            = mi8 + 8 * k;
        m->block_mi.bsize           = (BlockSize)r[0];
        m->block_mi.tx_depth        = r[1];
        m->block_mi.skip            = r[2];
        m->block_mi.ref_frame[0]    = (MvReferenceFrame)(int8_t)r[3];
        m->block_mi.mode            = (PredictionMode)r[4];
        m->block_mi.segment_id      = r[5];
        m->cdef_strength            = 0;
        grid[k]                     = (ModeInfo *)m;
    }
    pcs->mi_grid_base = grid;
    pcs->mi_stride    = (uint16_t)mi_cols;
    /* pictures: recon (the encoder's EncDec output) and source */
    EbPictureBufferDesc *recon, *input;
    if (new_pic(&recon, W, H, hbd, 96) || new_pic(&input, W, H, hbd, 96)) return 1;
    for (int p = 0; p < 3; p++) {
        const int w = p ? W / 2 : W, h = p ? H / 2 : H;
        const size_t o = p == 0 ? 0 : p == 1 ? ny : ny + nc;
        put_pic(recon, p, rec + o, w, h);
        put_pic(input, p, src + o, w, h);
    }
    if (hbd) {
        eds->recon_pic_16bit   = recon;
        pcs->input_frame16bit  = input;
        EbPictureBufferDesc *e = calloc(1, sizeof(*e)); /* read only for its bit depth (lambda assignment) */
        e->bit_depth           = EB_TEN_BIT;
        ppcs->enhanced_pic     = e;
    } else {
        eds->recon_pic              = recon;
        ppcs->enhanced_pic          = input;
        ppcs->enhanced_unscaled_pic = input;
    }

    GoldenFile g = golden_open(out_path);
    golden_put1(&g, "header", 'i', I_COUNT, hdr);

    /* ---- DLF (EbDlfProcess.c:96-106), or the SB-based DLF of the encode loop (EbCodingLoop.c:2260-2281) ---- */
    if (ppcs->dlf_ctrls.enabled && ppcs->dlf_ctrls.sb_based_dlf) {
        /* LPF_PICK_FROM_Q: no listed references (their levels never force 0), every SB's ME distortion = I_MESAD */
        pcs->slice_type        = (SliceType)hdr[I_SLICE_TYPE];
        ppcs->input_resolution = (EbInputResolution)hdr[I_IN_RES];
        ppcs->tot_ref_frame_types = 0;
        const int nsb64        = ((W + 63) / 64) * ((H + 63) / 64);
        pcs->b64_total_count   = (uint16_t)nsb64;
        ppcs->rc_me_distortion = calloc((size_t)nsb64, sizeof(uint32_t));
        for (int b = 0; b < nsb64; b++) ppcs->rc_me_distortion[b] = (uint32_t)hdr[I_MESAD];
        /* the encode loop's order: SBs in raster order, each filtered right after its own coding */
        for (int sy = 0; sy < H; sy += SB)
            for (int sx = 0; sx < W; sx += SB) {
                if (sx == 0 && sy == 0) {
                    svt_av1_loop_filter_init(pcs);
                    svt_av1_pick_filter_level(ppcs->enhanced_pic, pcs, LPF_PICK_FROM_Q);
                    svt_av1_loop_filter_frame_init(fh, &ppcs->lf_info, 0, 3);
                }
                if (lf->filter_level[0] || lf->filter_level[1]) {
                    const int sbw = SB < W - sx ? SB : W - sx;
                    svt_aom_loop_filter_sb(recon, pcs, sy >> 2, sx >> 2, 0, 3, (uint8_t)(sx + sbw == W));
                }
            }
    } else if (ppcs->dlf_ctrls.enabled) {
        svt_av1_loop_filter_init(pcs);
        svt_av1_pick_filter_level(ppcs->enhanced_pic, pcs, LPF_PICK_FROM_FULL_IMAGE);
        svt_av1_loop_filter_frame(recon, pcs, 0, 3);
    }
    const int32_t lfl[4] = {lf->filter_level[0], lf->filter_level[1], lf->filter_level_u, lf->filter_level_v};
    golden_put1(&g, "lf_levels", 'i', 4, lfl);
    emit_pic(&g, "dlf", recon, W, H);

    /* ---- pre-CDEF prep (EbDlfProcess.c:109-136) ---- */
    Yv12BufferConfig fts;
    memset(&fts, 0, sizeof fts);
    cm->frame_to_show = &fts;
    pcs->rst_info[0].restoration_unit_size = hdr[I_US_Y];
    pcs->rst_info[1].restoration_unit_size = pcs->rst_info[2].restoration_unit_size = hdr[I_US_UV];
    svt_av1_alloc_restoration_buffers(pcs, cm);
    svt_aom_link_eb_to_aom_buffer_desc(recon, cm->frame_to_show, 0, 0, hbd);
    svt_av1_loop_restoration_save_boundary_lines(cm->frame_to_show, cm, 0);
    for (int p = 0; p < 3; p++) {
        int st;
        pcs->cdef_input_recon[p]  = plane_ptr(recon, p, &st);
        pcs->cdef_input_source[p] = plane_ptr(input, p, &st);
    }

    /* ---- CDEF (EbCdefProcess.c:398-520) ---- */
    const int nvfb = (mi_rows + 15) / 16, nhfb = (mi_cols + 15) / 16, nfb = nvfb * nhfb;
    pcs->mse_seg[0]     = calloc((size_t)nfb, sizeof(*pcs->mse_seg[0]));
    pcs->mse_seg[1]     = calloc((size_t)nfb, sizeof(*pcs->mse_seg[1]));
    pcs->skip_cdef_seg  = calloc((size_t)nfb, 1);
    pcs->cdef_dir_data  = calloc((size_t)nfb, sizeof(CdefDirData));
    pcs->cdef_segments_column_count = (uint8_t)hdr[I_CDEF_SC];
    pcs->cdef_segments_row_count    = (uint8_t)hdr[I_CDEF_SR];
    const int nseg_cdef             = hdr[I_CDEF_SC] * hdr[I_CDEF_SR];
    uint32_t  fast_lambda = 0, full_lambda = 0;
    svt_aom_av1_lambda_assignment_function_table[ppcs->pred_structure](
        pcs, &fast_lambda, &full_lambda, (uint8_t)ppcs->enhanced_pic->bit_depth, fh->quantization_params.base_q_idx,
        FALSE);
    const uint64_t lam = full_lambda;
    golden_put1(&g, "cdef_lambda", 'Q', 1, &lam);
    int32_t applied = 0;
    if (scs->seq_header.cdef_level && ppcs->cdef_level) {
        if (!ppcs->cdef_ctrls.use_reference_cdef_fs)
            for (int s = 0; s < nseg_cdef; s++) ref_cdef_seg_search(pcs, scs, (uint32_t)s);
        finish_cdef_search(pcs);
        CdefParams *cp = &fh->cdef_params;
        if (cp->cdef_y_strength[0] != 0 || cp->cdef_uv_strength[0] != 0 || ppcs->nb_cdef_strengths != 1) {
            svt_av1_cdef_frame(scs, pcs);
            applied = 1;
        }
    }
    {
        CdefParams *cp      = &fh->cdef_params;
        int32_t     prm[20] = {cp->cdef_damping, cp->cdef_bits, ppcs->nb_cdef_strengths, applied};
        for (int k = 0; k < 8; k++) prm[4 + k] = cp->cdef_y_strength[k], prm[12 + k] = cp->cdef_uv_strength[k];
        golden_put1(&g, "cdef_params", 'i', 20, prm);
        uint64_t *mse = malloc(sizeof(uint64_t) * 2 * nfb * 64);
        /* dir / var: CDEF_NBLOCKS x CDEF_NBLOCKS (16 x 16) per filter block; a 128-block search fills all of it */
        uint8_t  *dir = malloc((size_t)nfb * 256);
        int32_t  *var = malloc(sizeof(int32_t) * nfb * 256);
        int8_t   *fbs = malloc((size_t)nfb);
        for (int f = 0; f < nfb; f++) {
            for (int k = 0; k < 64; k++) {
                mse[(size_t)f * 64 + k]         = pcs->mse_seg[0][f][k];
                mse[(size_t)(nfb + f) * 64 + k] = pcs->mse_seg[1][f][k];
            }
            for (int k = 0; k < 256; k++) {
                dir[(size_t)f * 256 + k] = pcs->cdef_dir_data[f].dir[k >> 4][k & 15];
                var[(size_t)f * 256 + k] = pcs->cdef_dir_data[f].var[k >> 4][k & 15];
            }
            const int fbr = f / nhfb, fbc = f % nhfb;
            fbs[f] = cells[(size_t)16 * fbr * mi_cols + 16 * fbc].cdef_strength;
        }
        uint32_t d3[3] = {2, (uint32_t)nfb, 64};
        golden_put(&g, "cdef_mse", 'Q', 3, d3, mse);
        golden_put1(&g, "cdef_skip", 'B', (uint32_t)nfb, pcs->skip_cdef_seg);
        golden_put2(&g, "cdef_dir", 'B', (uint32_t)nfb, 256, dir);
        golden_put2(&g, "cdef_var", 'i', (uint32_t)nfb, 256, var);
        golden_put1(&g, "cdef_fbs", 'b', (uint32_t)nfb, fbs);
        free(mse), free(dir), free(var), free(fbs);
    }
    emit_pic(&g, "cdef", recon, W, H);

    /* ---- restoration prep (EbCdefProcess.c:663-670) and search / apply (EbRestProcess.c:552-630) ---- */
    svt_av1_loop_restoration_save_boundary_lines(cm->frame_to_show, cm, 1);
    for (int p = 0; p < 3; p++)
        pcs->rusi_picture[p] = calloc((size_t)pcs->rst_info[p].units_per_tile, sizeof(RestUnitSearchInfo));
    pcs->rest_search_mutex          = svt_create_mutex();
    pcs->rest_segments_column_count = (uint8_t)hdr[I_REST_SC];
    pcs->rest_segments_row_count    = (uint8_t)hdr[I_REST_SR];
    pcs->rest_segments_total_count  = (uint16_t)(hdr[I_REST_SC] * hdr[I_REST_SR]);
    EbPictureBufferDesc *trial;
    if (new_pic(&trial, W, H, hbd, 96)) return 1;
    Yv12BufferConfig cpi_source, trial_frame_rst, org_fts;
    svt_aom_link_eb_to_aom_buffer_desc(input, &cpi_source, 0, 0, hbd);
    svt_aom_link_eb_to_aom_buffer_desc(trial, &trial_frame_rst, 0, 0, hbd);
    svt_aom_link_eb_to_aom_buffer_desc(recon, &org_fts, 0, 0, hbd);
    int32_t *tmpbuf = malloc(RESTORATION_TMPBUF_SIZE);
#ifndef SVTGPU_BIND
    g_rec.pic                    = recon; /* record the statistics the search computes (the C kernels, unchanged) */
    svt_av1_compute_stats        = rec_compute_stats;
    svt_av1_compute_stats_highbd = rec_compute_stats_highbd;
#endif
    for (int s = 0; s < pcs->rest_segments_total_count; s++)
        restoration_seg_search(tmpbuf, &org_fts, &cpi_source, &trial_frame_rst, pcs, (uint32_t)s);
    rest_finish_search(pcs);
#ifndef SVTGPU_BIND
    svt_av1_compute_stats        = svt_av1_compute_stats_c;
    svt_av1_compute_stats_highbd = svt_av1_compute_stats_highbd_c;
    if (g_rec.n) {
        golden_put2(&g, "wn_stats_meta", 'i', (uint32_t)g_rec.n, 6, g_rec.meta);
        golden_put1(&g, "wn_stats_M", 'q', (uint32_t)g_rec.nm, g_rec.M);
        golden_put1(&g, "wn_stats_H", 'q', (uint32_t)g_rec.nh, g_rec.H);
    }
#endif
    int32_t ft[3];
    for (int p = 0; p < 3; p++) ft[p] = pcs->rst_info[p].frame_restoration_type;
    if (ft[0] != RESTORE_NONE || ft[1] != RESTORE_NONE || ft[2] != RESTORE_NONE)
        svt_av1_loop_restoration_filter_frame(tmpbuf, cm->frame_to_show, cm, 0);
    golden_put1(&g, "lr_ftype", 'i', 3, ft);
    for (int p = 0; p < 3; p++) {
        const RestorationInfo *rsi = &pcs->rst_info[p];
        const int              nu  = rsi->units_per_tile;
        int32_t               *u   = calloc((size_t)nu, 20 * sizeof(int32_t));
        int64_t               *ss  = calloc((size_t)nu, 3 * sizeof(int64_t));
        int32_t               *sp  = calloc((size_t)nu, 19 * sizeof(int32_t));
        for (int k = 0; k < nu; k++) {
            const RestorationUnitInfo *ui = &rsi->unit_info[k];
            int32_t                   *e  = u + 20 * k;
            e[0]                          = ft[p] == RESTORE_NONE ? 0 : ui->restoration_type;
            /* the parameters of the unit's own type only: the reference leaves the others' fields unwritten (their
             * bytes differ from run to run), so they are stored as zeros and the fixtures are reproducible */
            if (e[0] == RESTORE_WIENER)
                for (int q = 0; q < 8; q++) e[1 + q] = ui->wiener_info.vfilter[q], e[9 + q] = ui->wiener_info.hfilter[q];
            if (e[0] == RESTORE_SGRPROJ)
                e[17] = ui->sgrproj_info.ep, e[18] = ui->sgrproj_info.xqd[0], e[19] = ui->sgrproj_info.xqd[1];
            const RestUnitSearchInfo *rs = &pcs->rusi_picture[p][k];
            for (int q = 0; q < 3; q++) ss[3 * k + q] = rs->sse[q] == INT64_MAX ? -1 : rs->sse[q];
            if (rs->sse[1] != INT64_MAX)
                for (int q = 0; q < 8; q++) sp[19 * k + q] = rs->wiener.vfilter[q], sp[19 * k + 8 + q] = rs->wiener.hfilter[q];
            if (rs->sse[2] != INT64_MAX)
                sp[19 * k + 16] = rs->sgrproj.ep, sp[19 * k + 17] = rs->sgrproj.xqd[0], sp[19 * k + 18] = rs->sgrproj.xqd[1];
        }
        char nm[32];
        snprintf(nm, sizeof nm, "lr_units%d", p);
        golden_put2(&g, nm, 'i', (uint32_t)nu, 20, u);
        snprintf(nm, sizeof nm, "lr_sse%d", p);
        golden_put2(&g, nm, 'q', (uint32_t)nu, 3, ss);
        snprintf(nm, sizeof nm, "lr_rec%d", p);
        golden_put2(&g, nm, 'i', (uint32_t)nu, 19, sp);
        free(u), free(ss), free(sp);
    }
    emit_pic(&g, "lr", recon, W, H);
    golden_close(&g);
    free(tmpbuf);
    free(in);
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* svt_av1_pick_filter_level(LPF_PICK_FROM_Q) (EbDeblockingFilter.c:1036-1138) and qp_based_dlf_param (:991)     */
/* ------------------------------------------------------------------------------------------- */
#define BYQ_N 640
#define BYQ_IN 24
static int run_byq(const char *out_path) {
    Rng                      r    = {0xD1F0000000000B79ull};
    SequenceControlSet      *scs  = calloc(1, sizeof(*scs));
    PictureParentControlSet *ppcs = calloc(1, sizeof(*ppcs));
    PictureControlSet       *pcs  = calloc(1, sizeof(*pcs));
    pcs->scs = ppcs->scs = scs;
    pcs->ppcs            = ppcs;
    EbReferenceObject refs[8];
    EbObjectWrapper   wraps[8];
    memset(refs, 0, sizeof refs);
    memset(wraps, 0, sizeof wraps);
    static const uint8_t list_of[8] = {0, 0, 0, 0, 0, 1, 1, 1}, idx_of[8] = {0, 0, 1, 2, 3, 0, 1, 2};
    for (int t = 1; t < 8; t++) {
        wraps[t].object_ptr                      = &refs[t];
        pcs->ref_pic_ptr_array[list_of[t]][idx_of[t]] = &wraps[t];
    }
    uint32_t *me_sad = calloc(4096, sizeof(uint32_t));
    ppcs->rc_me_distortion = me_sad;
    /* per case: in {bd, q, frame_type, slice_type, tl_pcs, tl_ppcs, in_res, zero_lvl, nsb, nref, ref types[4],
     *              me_sad seed value, me spread, lvl y0 y1 u v of each listed ref packed: 4 x 4 bytes} */
    int32_t *vin  = calloc(BYQ_N, BYQ_IN * sizeof(int32_t));
    int32_t *vout = calloc(BYQ_N, 6 * sizeof(int32_t));
    uint32_t *sads = calloc((size_t)BYQ_N * 64, sizeof(uint32_t));
    for (int n = 0; n < BYQ_N; n++) {
        int32_t  *v  = vin + BYQ_IN * n;
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12;
        v[0] = bd;
        v[1] = n < 12 ? n * 23 : (int)rng_below(&r, 256);
        v[2] = rng_below(&r, 4) == 0 ? KEY_FRAME : INTER_FRAME;
        v[3] = v[2] == KEY_FRAME ? I_SLICE : (rng_below(&r, 3) == 0 ? P_SLICE : B_SLICE);
        if (rng_below(&r, 8) == 0) v[3] = I_SLICE;
        v[4] = (int)rng_below(&r, 6);
        v[5] = rng_below(&r, 4) == 0 ? (int)rng_below(&r, 6) : v[4];
        v[6] = (int)rng_below(&r, INPUT_SIZE_COUNT);
        v[7] = (int)rng_below(&r, 4);
        v[8] = 1 + (int)rng_below(&r, 64);
        v[9] = (int)rng_below(&r, 5);
        for (int k = 0; k < 4; k++) {
            /* single references 1..7, now and then a compound pair (skipped by the reference) */
            v[10 + k] = rng_below(&r, 6) == 0 ? TOTAL_REFS_PER_FRAME + (int)rng_below(&r, 8) : 1 + (int)rng_below(&r, 7);
        }
        const uint32_t base = rng_below(&r, 4) == 0 ? (uint32_t)rng_next(&r) : rng_below(&r, 40000);
        for (int b = 0; b < v[8]; b++) sads[(size_t)n * 64 + b] = base + rng_below(&r, 1 + base / 2 + 100);
        for (int k = 0; k < 4; k++) {
            const int lo = rng_below(&r, 5) == 0 ? 0 : (int)rng_below(&r, 64);
            uint32_t  pk = 0;
            for (int j = 0; j < 4; j++) {
                const uint32_t lv = rng_below(&r, 6) == 0 ? 0u : (uint32_t)((lo + (int)rng_below(&r, 8)) % 64);
                pk |= lv << (8 * j);
            }
            v[14 + k] = (int32_t)pk;
        }
        /* apply */
        scs->static_config.encoder_bit_depth       = (uint32_t)bd;
        ppcs->frm_hdr.quantization_params.base_q_idx = (uint8_t)v[1];
        ppcs->frm_hdr.frame_type                   = (FrameType)v[2];
        pcs->slice_type                            = (SliceType)v[3];
        pcs->temporal_layer_index                  = (uint8_t)v[4];
        ppcs->temporal_layer_index                 = (uint8_t)v[5];
        ppcs->input_resolution                     = (EbInputResolution)v[6];
        ppcs->dlf_ctrls.zero_filter_strength_lvl   = (uint8_t)v[7];
        pcs->b64_total_count                       = (uint16_t)v[8];
        memcpy(me_sad, sads + (size_t)n * 64, sizeof(uint32_t) * 64);
        ppcs->tot_ref_frame_types = (uint8_t)v[9];
        for (int k = 0; k < 4; k++) ppcs->ref_frame_type_arr[k] = (MvReferenceFrame)v[10 + k];
        for (int t = 1; t < 8; t++) refs[t].filter_level[0] = refs[t].filter_level[1] = refs[t].filter_level_u =
                                        refs[t].filter_level_v = 63;
        for (int k = 0; k < v[9]; k++) {
            const int t = v[10 + k];
            if (t >= TOTAL_REFS_PER_FRAME) continue;
            const uint32_t pk = (uint32_t)v[14 + k];
            refs[t].filter_level[0] = (int32_t)(pk & 255), refs[t].filter_level[1] = (int32_t)((pk >> 8) & 255);
            refs[t].filter_level_u = (int32_t)((pk >> 16) & 255), refs[t].filter_level_v = (int32_t)(pk >> 24);
        }
        ppcs->frm_hdr.loop_filter_params.filter_level[0] = ppcs->frm_hdr.loop_filter_params.filter_level[1] = -1;
        svt_av1_pick_filter_level(NULL, pcs, LPF_PICK_FROM_Q);
        const struct LoopFilter *lf = &ppcs->frm_hdr.loop_filter_params;
        int32_t                 *o  = vout + 6 * n;
        o[0] = lf->filter_level[0], o[1] = lf->filter_level[1], o[2] = lf->filter_level_u, o[3] = lf->filter_level_v;
        qp_based_dlf_param(pcs, &o[4], &o[5]);
    }
    GoldenFile g = golden_open(out_path);
    golden_put2(&g, "in", 'i', BYQ_N, BYQ_IN, vin);
    golden_put2(&g, "me_sad", 'I', BYQ_N, 64, sads);
    golden_put2(&g, "out", 'i', BYQ_N, 6, vout);
    /* the AC quantizer the level guess is fitted on (svt_aom_ac_quant_qtx, EbInvTransforms.c:3379) */
    int32_t acq[3 * 256];
    for (int b = 0; b < 3; b++)
        for (int q = 0; q < 256; q++) acq[256 * b + q] = svt_aom_ac_quant_qtx(q, 0, (EbBitDepth)(8 + 2 * b));
    golden_put2(&g, "ac_quant", 'i', 3, 256, acq);
    golden_close(&g);
    free(vin), free(vout), free(sads), free(me_sad);
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* control tables of every level (EncModeConfig.c:860 / :1329 / :1386 / :1557)                  */
/* ------------------------------------------------------------------------------------------- */
static int run_ctrls(const char *out_path) {
    GoldenFile               g    = golden_open(out_path);
    PictureParentControlSet *ppcs = calloc(1, sizeof(*ppcs));
    Av1Common               *cm   = calloc(1, sizeof(*cm));
    /* cdef: per level {enabled, first_pass_fs_num, default_second_pass_fs_num, use_reference_cdef_fs,
     * search_best_ref_fs, subsampling_factor, zero_fs_cost_bias, use_skip_detector} + fs[64] + fs2[64] +
     * fs_uv[64] + fs2_uv[64] */
    const int NC = 18, CW = 8 + 4 * 64;
    int32_t  *c  = calloc((size_t)NC * CW, sizeof(int32_t));
    for (int l = 0; l < NC; l++) {
        memset(&ppcs->cdef_ctrls, 0, sizeof ppcs->cdef_ctrls);
        ref_set_cdef_controls(ppcs, (uint8_t)l, 0);
        const CdefControls *cc = &ppcs->cdef_ctrls;
        int32_t            *e  = c + (size_t)CW * l;
        e[0] = cc->enabled, e[1] = cc->first_pass_fs_num, e[2] = cc->default_second_pass_fs_num;
        e[3] = cc->use_reference_cdef_fs, e[4] = cc->search_best_ref_fs, e[5] = cc->subsampling_factor;
        e[6] = cc->zero_fs_cost_bias, e[7] = cc->use_skip_detector;
        for (int k = 0; k < 64; k++) {
            e[8 + k]       = cc->default_first_pass_fs[k];
            e[8 + 64 + k]  = cc->default_second_pass_fs[k];
            e[8 + 128 + k] = cc->default_first_pass_fs_uv[k];
            e[8 + 192 + k] = cc->default_second_pass_fs_uv[k];
        }
    }
    golden_put2(&g, "cdef", 'i', (uint32_t)NC, (uint32_t)CW, c);
    int32_t d[6 * 6];
    for (int l = 0; l < 6; l++) {
        memset(&ppcs->dlf_ctrls, 0, sizeof ppcs->dlf_ctrls);
        ref_set_dlf_controls(ppcs, (uint8_t)l);
        const DlfCtrls *dc = &ppcs->dlf_ctrls;
        int32_t        *e  = d + 6 * l;
        e[0] = dc->enabled, e[1] = dc->sb_based_dlf, e[2] = dc->dlf_avg, e[3] = dc->dlf_avg_uv;
        e[4] = dc->early_exit_convergence, e[5] = dc->zero_filter_strength_lvl;
    }
    golden_put2(&g, "dlf", 'i', 6, 6, d);
    int32_t w[6 * 6];
    for (int l = 0; l < 6; l++) {
        memset(&cm->wn_filter_ctrls, 0, sizeof cm->wn_filter_ctrls);
        ref_set_wn_filter_ctrls(cm, (uint8_t)l);
        const WnFilterCtrls *wc = &cm->wn_filter_ctrls;
        int32_t             *e  = w + 6 * l;
        e[0] = wc->enabled, e[1] = wc->filter_tap_lvl, e[2] = wc->use_refinement, e[3] = wc->max_one_refinement_step;
        e[4] = wc->use_prev_frame_coeffs, e[5] = wc->use_chroma;
    }
    golden_put2(&g, "wn", 'i', 6, 6, w);
    int32_t s[5 * 11];
    for (int l = 0; l < 5; l++) {
        memset(&cm->sg_filter_ctrls, 0, sizeof cm->sg_filter_ctrls);
        ref_set_sg_filter_ctrls(cm, (uint8_t)l);
        const SgFilterCtrls *sc = &cm->sg_filter_ctrls;
        int32_t             *e  = s + 11 * l;
        e[0] = sc->enabled, e[1] = sc->step_range, e[2] = sc->use_chroma;
        for (int k = 0; k < 2; k++)
            e[3 + k] = sc->start_ep[k], e[5 + k] = sc->end_ep[k], e[7 + k] = sc->ep_inc[k], e[9 + k] = sc->refine[k];
    }
    golden_put2(&g, "sg", 'i', 5, 11, s);
    golden_close(&g);
    return 0;
}

int main(int argc, char **argv) {
    bind_c_kernels();
#ifdef SVTGPU_BIND
    if (!svtgpu_device_available()) {
        fprintf(stderr, "rtcd_pipe: no gfx950 device\n");
        return 3;
    }
    bind_device_kernels();
#endif
    if (argc == 4 && !strcmp(argv[1], "pipe")) return run_pipe(argv[2], argv[3]);
    if (argc == 3 && !strcmp(argv[1], "byq")) return run_byq(argv[2]);
    if (argc == 3 && !strcmp(argv[1], "ctrls")) return run_ctrls(argv[2]);
    fprintf(stderr, "usage: %s pipe <in> <out> | byq <out> | ctrls <out>\n", argv[0]);
    return 2;
}
