/*
 * ref_bench.c — the REFERENCE's CPU path timed on the bench workload (test infrastructure: bench.py's
 * cpu_baseline, kind "reference"; never shipped).
 *
 * Links the reference's own C and its AVX2/SSE2 kernels (compiled from /root/reference by oracle/ref.mk) with the
 * RTCD pointers bound the way svt_aom_setup_rtcd_internal / svt_aom_setup_common_rtcd_internal bind them on an
 * AVX2 host (common_dsp_rtcd.c:309-311, 352, 626-658; aom_dsp_rtcd.c:184-208, 478, 499), and runs the stages of
 * bench.py's GPU step on crops of the same frame, one crop per thread at a time (the encoder's own parallelism is
 * per segment / picture; independent crops bound it from above):
 *   DLF     search_filter_level's bisection (EbDeblockingFilter.c:886-991) over svt_av1_loop_filter_frame trials +
 *           the frame SSE, then the frame filter;
 *   CDEF    cdef_seg_search's FB loop (EbCdefProcess.c:114-357: svt_cdef_filter_fb + compute_cdef_dist over the 64
 *           strengths), finish_cdef_search's strength selection (EbEncCdef.c:697-890, svt_search_one_dual), the
 *           apply (svt_cdef_filter_fb per FB, unfiltered neighbours);
 *   LR      restoration_seg_search + rest_finish_search + svt_av1_loop_restoration_filter_frame;
 *   MD      SAD (svt_aom_sad_16bit_kernel_avx2), SSE (svt_aom_highbd_sse_avx2) and variance
 *           (svt_aom_variance_highbd_c: the reference has no SIMD version of it; svt_aom_highbd_sse_avx2 takes plain
 *           uint16_t pointers, sse_avx2.c:75-80) of every block shape <= 64x64 of
 *           every SB against every reference at its MV.
 * The restated loops are the reference's control flow around its own kernels; the outputs are not checked here
 * (the oracle and the GPU path are, against the reference's goldens).
 *
 * usage: ref_bench <input.bin> <threads> [passes]   (input written by bench.py: header, CDEF controls, planes, mi, refs,
 *        MVs; every pass runs every crop once)
 *        REF_BENCH_STAGES = bit mask of the stages run (1 DLF, 2 CDEF search + pick + apply, 4 LR, 8 MD; default 15);
 *        8-bit input runs the CDEF stage alone on the reference's 8-bit path
 *        (is_16bit_pipeline = 0: svt_aom_copy_sb8_16 from 8-bit recon, svt_compute_cdef_dist_8bit, 8-bit apply).
 * prints: ref_bench px=<luma pixels> seconds=<wall> threads=<T>
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "EbDefinitions.h"
#include "EbPictureControlSet.h"
#include "EbSequenceControlSet.h"
#include "EbDeblockingFilter.h"
#include "EbRestoration.h"
#include "EbCdef.h"
#include "Av1Common.h"
#include "EbCodingUnit.h"
#include "EbThreads.h"
#include "common_dsp_rtcd.h"
#include "aom_dsp_rtcd.h"
#include "../../include/svtgpu.h"

void    svt_av1_loop_filter_init(PictureControlSet *pcs);
void    svt_av1_loop_filter_frame(EbPictureBufferDesc *frame_buffer, PictureControlSet *pcs, int32_t plane_start,
                                  int32_t plane_end);
void    svt_av1_loop_restoration_filter_frame(int32_t *rst_tmpbuf, Yv12BufferConfig *frame, Av1Common *cm,
                                              int32_t optimized_lr);
void    svt_av1_loop_restoration_save_boundary_lines(const Yv12BufferConfig *frame, Av1Common *cm, int32_t after_cdef);
int32_t svt_aom_realloc_frame_buffer(Yv12BufferConfig *ybf, int32_t width, int32_t height, int32_t ss_x, int32_t ss_y,
                                     int32_t use_highbitdepth, int32_t border, int32_t byte_alignment,
                                     AomCodecFrameBuffer *fb, AomGetFrameBufferCbFn cb, void *cb_priv);
EbErrorType svt_av1_alloc_restoration_buffers(PictureControlSet *pcs, Av1Common *cm);
void        restoration_seg_search(int32_t *rst_tmpbuf, Yv12BufferConfig *org_fts, const Yv12BufferConfig *src,
                                   Yv12BufferConfig *trial_frame_rst, PictureControlSet *pcs, uint32_t segment_index);
void        rest_finish_search(PictureControlSet *pcs);
int32_t     svt_sb_compute_cdef_list(PictureControlSet *pcs, const Av1Common *const cm, int32_t mi_row, int32_t mi_col,
                                     CdefList *dlist, BlockSize bs);
/* AVX2 / SSE2 kernels (reference ASM_AVX2 / ASM_SSE2 sources) */
uint8_t  svt_aom_cdef_find_dir_avx2(const uint16_t *img, int32_t stride, int32_t *var, int32_t coeff_shift);
void     svt_aom_cdef_find_dir_dual_avx2(const uint16_t *img1, const uint16_t *img2, int stride, int32_t *var1,
                                         int32_t *var2, int32_t coeff_shift, uint8_t *out1, uint8_t *out2);
void     svt_cdef_filter_block_avx2(uint8_t *dst8, uint16_t *dst16, int32_t dstride, const uint16_t *in, int32_t pri,
                                    int32_t sec, int32_t dir, int32_t pri_damping, int32_t sec_damping, int32_t bsize,
                                    int32_t coeff_shift, uint8_t subsampling_factor);
void     svt_cdef_filter_block_8xn_16_avx2(const uint16_t *const in, const int32_t pri_strength,
                                           const int32_t sec_strength, const int32_t dir, int32_t pri_damping,
                                           int32_t sec_damping, const int32_t coeff_shift, uint16_t *const dst,
                                           const int32_t dstride, uint8_t height, uint8_t subsampling_factor);
uint64_t svt_aom_compute_cdef_dist_16bit_avx2(const uint16_t *dst, int32_t dstride, const uint16_t *src,
                                              const CdefList *dlist, int32_t cdef_count, BlockSize bsize,
                                              int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
uint64_t svt_aom_compute_cdef_dist_8bit_avx2(const uint8_t *dst8, int32_t dstride, const uint8_t *src8,
                                             const CdefList *dlist, int32_t cdef_count, BlockSize bsize,
                                             int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
void     svt_aom_copy_rect8_8bit_to_16bit_avx2(uint16_t *dst, int32_t dstride, const uint8_t *src, int32_t sstride,
                                               int32_t v, int32_t h);
uint64_t svt_search_one_dual_avx2(int *lev0, int *lev1, int nb_strengths, uint64_t **mse[2], int sb_count,
                                  int start_gi, int end_gi);
uint64_t svt_full_distortion_kernel16_bits_avx2(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                                uint8_t *pred, int32_t pred_offset, uint32_t pred_stride,
                                                uint32_t area_width, uint32_t area_height);
uint32_t svt_aom_sad_16bit_kernel_avx2(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride,
                                       uint32_t height, uint32_t width);
int64_t  svt_aom_highbd_sse_avx2(const uint8_t *a8, int a_stride, const uint8_t *b8, int b_stride, int width, int height);
uint32_t svt_aom_variance_highbd_c(const uint16_t *a, int a_stride, const uint16_t *b, int b_stride, int w, int h,
                                   uint32_t *sse);

static void bind_kernels(void) {
    /* C first (everything the stages may reach), then the AVX2/SSE2 versions an AVX2 host gets */
    svt_memcpy                             = svt_memcpy_c;
    svt_log2f                              = svt_aom_log2f_32;
    svt_aom_lpf_horizontal_4               = svt_aom_lpf_horizontal_4_sse2;
    svt_aom_lpf_horizontal_6               = svt_aom_lpf_horizontal_6_sse2;
    svt_aom_lpf_horizontal_8               = svt_aom_lpf_horizontal_8_sse2;
    svt_aom_lpf_horizontal_14              = svt_aom_lpf_horizontal_14_sse2;
    svt_aom_lpf_vertical_4                 = svt_aom_lpf_vertical_4_sse2;
    svt_aom_lpf_vertical_6                 = svt_aom_lpf_vertical_6_sse2;
    svt_aom_lpf_vertical_8                 = svt_aom_lpf_vertical_8_sse2;
    svt_aom_lpf_vertical_14                = svt_aom_lpf_vertical_14_sse2;
    svt_aom_highbd_lpf_horizontal_4        = svt_aom_highbd_lpf_horizontal_4_sse2;
    svt_aom_highbd_lpf_horizontal_6        = svt_aom_highbd_lpf_horizontal_6_sse2;
    svt_aom_highbd_lpf_horizontal_8        = svt_aom_highbd_lpf_horizontal_8_sse2;
    svt_aom_highbd_lpf_horizontal_14       = svt_aom_highbd_lpf_horizontal_14_sse2;
    svt_aom_highbd_lpf_vertical_4          = svt_aom_highbd_lpf_vertical_4_sse2;
    svt_aom_highbd_lpf_vertical_6          = svt_aom_highbd_lpf_vertical_6_sse2;
    svt_aom_highbd_lpf_vertical_8          = svt_aom_highbd_lpf_vertical_8_sse2;
    svt_aom_highbd_lpf_vertical_14         = svt_aom_highbd_lpf_vertical_14_sse2;
    svt_cdef_filter_block                  = svt_cdef_filter_block_avx2;
    svt_cdef_filter_block_8xn_16           = svt_cdef_filter_block_8xn_16_avx2;
    svt_aom_cdef_find_dir                  = svt_aom_cdef_find_dir_avx2;
    svt_aom_cdef_find_dir_dual             = svt_aom_cdef_find_dir_dual_avx2;
    svt_compute_cdef_dist_16bit            = svt_aom_compute_cdef_dist_16bit_avx2;
    svt_compute_cdef_dist_8bit             = svt_aom_compute_cdef_dist_8bit_avx2;
    svt_search_one_dual                    = svt_search_one_dual_avx2;
    svt_aom_copy_rect8_8bit_to_16bit       = svt_aom_copy_rect8_8bit_to_16bit_avx2;
    svt_av1_wiener_convolve_add_src        = svt_av1_wiener_convolve_add_src_avx2;
    svt_av1_highbd_wiener_convolve_add_src = svt_av1_highbd_wiener_convolve_add_src_avx2;
    svt_av1_selfguided_restoration         = svt_av1_selfguided_restoration_avx2;
    svt_apply_selfguided_restoration       = svt_apply_selfguided_restoration_avx2;
    svt_av1_compute_stats                  = svt_av1_compute_stats_avx2;
    svt_av1_compute_stats_highbd           = svt_av1_compute_stats_highbd_avx2;
    svt_get_proj_subspace                  = svt_get_proj_subspace_c; /* its AVX2 version calls RunEmms (NASM) */
    svt_av1_lowbd_pixel_proj_error         = svt_av1_lowbd_pixel_proj_error_avx2;
    svt_av1_highbd_pixel_proj_error        = svt_av1_highbd_pixel_proj_error_avx2;
    svt_aom_mse16x16                       = svt_aom_mse16x16_avx2;
    svt_aom_highbd_8_mse16x16              = svt_aom_highbd_8_mse16x16_c;
}

/* ------------------------------------------------------------------------------------------- input */
enum { H_W, H_H, H_BD, H_NREF, H_Q, H_LAMBDA, H_GX, H_GY, H_RDMULT, H_SW0, H_SW1, H_SW2, H_WN0, H_WN1, H_SG0, H_SG1,
       H_LF0, H_LF1, H_LFU, H_LFV, H_N };
static int32_t            hdr[H_N];
static SvtGpuCdefControls cctl;
static uint16_t          *g_src[3], *g_rec[3], **g_ref;
static SvtGpuLfMi        *g_mi;
static int32_t           *g_mv; /* [nsb][nref][2] over the whole frame */

static void *xmalloc(size_t n) {
    void *p = calloc(1, n);
    if (!p) {
        fprintf(stderr, "ref_bench: out of memory\n");
        exit(1);
    }
    return p;
}

static void read_all(FILE *f, void *p, size_t n) {
    if (fread(p, 1, n, f) != n) {
        fprintf(stderr, "ref_bench: short input\n");
        exit(1);
    }
}

/* ------------------------------------------------------------------------------------------- one crop */
typedef struct Crop {
    int w, h, x0, y0; /* luma size and origin in the frame */
} Crop;

static uint16_t *crop_plane(uint16_t *const *planes, int p, const Crop *c) {
    const int W = hdr[H_W] >> (p > 0), pw = c->w >> (p > 0), ph = c->h >> (p > 0);
    const int x0 = c->x0 >> (p > 0), y0 = c->y0 >> (p > 0);
    uint16_t *o  = xmalloc(sizeof(uint16_t) * pw * ph);
    for (int y = 0; y < ph; y++) memcpy(o + (size_t)y * pw, planes[p] + (size_t)(y0 + y) * W + x0, 2 * pw);
    return o;
}

static int bsize_of(int w, int h) {
    for (int b = 0; b < BlockSizeS_ALL; b++)
        if (block_size_wide[b] == w && block_size_high[b] == h) return b;
    return -1;
}

static uint64_t plane_sse(uint16_t *a, uint16_t *b, int w, int h) {
    return svt_full_distortion_kernel16_bits_avx2((uint8_t *)a, 0, w, (uint8_t *)b, 0, w, w, h);
}

/* search_filter_level (EbDeblockingFilter.c:886-991) with try_filter_frame (:841-883): every trial filters a copy
 * of the plane and measures its SSE against the source */
static int dlf_search(PictureControlSet *pcs, EbPictureBufferDesc *trial, uint16_t *const *rec, uint16_t *const *src,
                      const int *last, int plane, int dir, int w, int h) {
    FrameHeader *fh = &pcs->ppcs->frm_hdr;
    const int    pw = w >> (plane > 0), ph = h >> (plane > 0);
    uint16_t    *tp = plane == 0 ? (uint16_t *)trial->buffer_y : plane == 1 ? (uint16_t *)trial->buffer_cb
                                                                             : (uint16_t *)trial->buffer_cr;
    int64_t      ss_err[MAX_LOOP_FILTER + 1];
    memset(ss_err, 0xFF, sizeof ss_err);
#define TRY(lvl)                                                                                                \
    ({                                                                                                          \
        int l_ = (lvl);                                                                                         \
        if (plane == 0) {                                                                                       \
            fh->loop_filter_params.filter_level[0] = dir == 1 ? fh->loop_filter_params.filter_level[0] : l_;    \
            fh->loop_filter_params.filter_level[1] = dir == 0 ? fh->loop_filter_params.filter_level[1] : l_;    \
        } else if (plane == 1)                                                                                  \
            fh->loop_filter_params.filter_level_u = l_;                                                         \
        else                                                                                                    \
            fh->loop_filter_params.filter_level_v = l_;                                                         \
        memcpy(tp, rec[plane], 2 * (size_t)pw * ph);                                                            \
        svt_av1_loop_filter_frame(trial, pcs, plane, plane + 1);                                                \
        (int64_t) plane_sse(tp, src[plane], pw, ph);                                                            \
    })
    int lvl = plane == 0 ? last[dir] : last[plane + 1];
    int mid = lvl < 0 ? 0 : lvl > MAX_LOOP_FILTER ? MAX_LOOP_FILTER : lvl, step = mid < 16 ? 4 : mid / 4;
    int64_t best_err = TRY(mid);
    int     best = mid, direction = 0, conv = 0;
    ss_err[mid]  = best_err;
    while (step > 0) {
        const int hi = AOMMIN(mid + step, MAX_LOOP_FILTER), lo = AOMMAX(mid - step, 0);
        int64_t   bias = (best_err >> (15 - (mid / 8))) * step;
        bias >>= 1; /* tx_mode != ONLY_4X4 */
        if (direction <= 0 && lo != mid) {
            if (ss_err[lo] < 0) ss_err[lo] = TRY(lo);
            if (ss_err[lo] < best_err + bias) {
                if (ss_err[lo] < best_err) best_err = ss_err[lo];
                best = lo;
            }
        }
        if (direction >= 0 && hi != mid) {
            if (ss_err[hi] < 0) ss_err[hi] = TRY(hi);
            if (ss_err[hi] < best_err - bias) best_err = ss_err[hi], best = hi;
        }
        if (best == mid) {
            conv++;
            step = step / 2; /* early_exit_convergence 0: never reached */
            direction = 0;
        } else {
            direction = best < mid ? -1 : 1;
            mid       = best;
        }
    }
#undef TRY
    return best;
}

static void set_lr_ctrls(Av1Common *cm) { /* wn / sg filter level 1 (svt_aom_set_wn/sg_filter_ctrls) */
    WnFilterCtrls *w = &cm->wn_filter_ctrls;
    SgFilterCtrls *g = &cm->sg_filter_ctrls;
    memset(w, 0, sizeof *w);
    memset(g, 0, sizeof *g);
    w->enabled = 1, w->use_chroma = 1, w->filter_tap_lvl = 1, w->use_refinement = 1, w->max_one_refinement_step = 0;
    g->enabled = 1, g->use_chroma = 1, g->step_range = 16;
    g->start_ep[0] = 0, g->end_ep[0] = 16, g->ep_inc[0] = 1;
    g->start_ep[1] = 0, g->end_ep[1] = 16, g->ep_inc[1] = 1;
    g->refine[0] = 1, g->refine[1] = 1;
}

static void to_y12(Yv12BufferConfig *f, uint16_t *const *pl, int w, int h) {
    for (int p = 0; p < 3; p++) {
        const int pw = w >> (p > 0), ph = h >> (p > 0), st = f->strides[p > 0];
        for (int y = 0; y < ph; y++)
            memcpy(CONVERT_TO_SHORTPTR(f->buffers[p]) + (size_t)y * st, pl[p] + (size_t)y * pw, 2 * (size_t)pw);
    }
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
static double          g_stage[5]; /* summed over threads: DLF, CDEF search, CDEF pick + apply, LR, MD */
static pthread_mutex_t g_stage_lock = PTHREAD_MUTEX_INITIALIZER;
static int             g_verbose;
static int             g_stages = 15;

static uint8_t *to8(const uint16_t *p, size_t n) { /* an 8-bit plane of the crop (the 8-bit pipeline's buffers) */
    uint8_t *o = xmalloc(n);
    for (size_t i = 0; i < n; i++) o[i] = (uint8_t)p[i];
    return o;
}

static void run_crop(const Crop *c, int32_t *tmpbuf) {
    double ts[6];
    ts[0] = now();
    const int W = c->w, H = c->h, bd = hdr[H_BD], cs = bd - 8, q = hdr[H_Q];
    uint16_t *src[3], *rec[3], *trl[3], *cdf[3];
    for (int p = 0; p < 3; p++) {
        src[p] = crop_plane(g_src, p, c);
        rec[p] = crop_plane(g_rec, p, c);
        trl[p] = xmalloc(2 * (size_t)(W >> (p > 0)) * (H >> (p > 0)));
    }
    /* ---- picture control structures and the mode-info grid of the crop ---- */
    SequenceControlSet      *scs  = xmalloc(sizeof *scs);
    PictureParentControlSet *ppcs = xmalloc(sizeof *ppcs);
    PictureControlSet       *pcs  = xmalloc(sizeof *pcs);
    Av1Common               *cm   = xmalloc(sizeof *cm);
    Macroblock              *x    = xmalloc(sizeof *x);
    pcs->scs = scs, pcs->ppcs = ppcs, ppcs->scs = scs, ppcs->av1_cm = cm, ppcs->av1x = x, cm->child_pcs = pcs;
    scs->sb_size = 64, scs->seq_header.sb_size = BLOCK_64X64, scs->is_16bit_pipeline = 1;
    scs->static_config.encoder_bit_depth = (uint32_t)bd;
    scs->max_input_luma_width = (uint16_t)W, scs->max_input_luma_height = (uint16_t)H;
    ppcs->aligned_width = (uint16_t)W, ppcs->aligned_height = (uint16_t)H;
    FrameHeader *fh = &ppcs->frm_hdr;
    fh->quantization_params.base_q_idx = (uint16_t)q;
    static const int8_t def_ref[8] = {1, 0, 0, 0, -1, 0, -1, -1};
    for (int k = 0; k < 8; k++) fh->loop_filter_params.ref_deltas[k] = def_ref[k];
    const int mi_cols = W >> 2, mi_rows = H >> 2, Wmi = hdr[H_W] >> 2;
    MbModeInfo *blocks = xmalloc(sizeof(MbModeInfo) * mi_rows * mi_cols);
    ModeInfo  **cells  = xmalloc(sizeof(ModeInfo *) * mi_rows * mi_cols);
    for (int r = 0; r < mi_rows; r++)
        for (int k = 0; k < mi_cols; k++) {
            const SvtGpuLfMi *m  = &g_mi[(size_t)((c->y0 >> 2) + r) * Wmi + (c->x0 >> 2) + k];
            const int         bw = block_size_wide[m->bsize] >> 2, bh = block_size_high[m->bsize] >> 2;
            const int         r0 = r - r % bh, k0 = k - k % bw; /* the block's top-left cell owns its record */
            MbModeInfo       *b  = &blocks[r0 * mi_cols + k0];
            if (r == r0 && k == k0) {
                b->block_mi.bsize        = (BlockSize)m->bsize;
                b->block_mi.tx_depth     = m->tx_depth;
                b->block_mi.skip         = m->skip;
                b->block_mi.ref_frame[0] = (MvReferenceFrame)m->ref_frame0;
                b->block_mi.mode         = (PredictionMode)m->mode;
                b->block_mi.segment_id   = m->segment_id;
            }
            cells[r * mi_cols + k] = (ModeInfo *)b;
        }
    pcs->mi_grid_base = cells, pcs->mi_stride = (uint16_t)mi_cols;
    cm->mi_rows = mi_rows, cm->mi_cols = mi_cols, cm->mi_stride = mi_cols;
    /* ---- DLF: level search (Y both directions, U, V) and the frame filter ---- */
    EbPictureBufferDesc pic, trial;
    memset(&pic, 0, sizeof pic);
    pic.bit_depth = bd > 8 ? EB_TEN_BIT : EB_EIGHT_BIT, pic.stride_y = (uint16_t)W;
    pic.stride_cb = pic.stride_cr = (uint16_t)(W / 2);
    trial = pic;
    pic.buffer_y = (uint8_t *)rec[0], pic.buffer_cb = (uint8_t *)rec[1], pic.buffer_cr = (uint8_t *)rec[2];
    trial.buffer_y = (uint8_t *)trl[0], trial.buffer_cb = (uint8_t *)trl[1], trial.buffer_cr = (uint8_t *)trl[2];
    svt_av1_loop_filter_init(pcs);
    const int last[4] = {hdr[H_LF0], hdr[H_LF1], hdr[H_LFU], hdr[H_LFV]}; /* the previous frame's levels */
    struct LoopFilter *lf = &fh->loop_filter_params;
    if (g_stages & 1) {
        lf->filter_level[0] = lf->filter_level[1] = dlf_search(pcs, &trial, rec, src, last, 0, 2, W, H);
        lf->filter_level_u = dlf_search(pcs, &trial, rec, src, last, 1, 0, W, H);
        lf->filter_level_v = dlf_search(pcs, &trial, rec, src, last, 2, 0, W, H);
        svt_av1_loop_filter_frame(&pic, pcs, 0, 3); /* rec[] is now the DLF output */
    }
    ts[1] = now();
    /* the 8-bit pipeline's planes (8-bit input: CDEF only) */
    const int is16 = bd > 8;
    uint8_t  *src8[3] = {NULL, NULL, NULL}, *rec8[3] = {NULL, NULL, NULL}, *cdf8[3] = {NULL, NULL, NULL};
    if (!is16)
        for (int p = 0; p < 3; p++) {
            const size_t n = (size_t)(W >> (p > 0)) * (H >> (p > 0));
            src8[p] = to8(src[p], n), rec8[p] = to8(rec[p], n), cdf8[p] = to8(rec[p], n);
        }
    /* ---- CDEF search: cdef_seg_search over the crop (one segment) ---- */
    const int nvfb = (mi_rows + 15) / 16, nhfb = (mi_cols + 15) / 16, nfb = nvfb * nhfb;
    const int nstr = cctl.first_pass_fs_num + cctl.default_second_pass_fs_num;
    uint64_t (*mse)[64] = xmalloc(sizeof(uint64_t) * 2 * nfb * 64); /* [2 * nfb][64] */
    uint8_t  *skipfb    = xmalloc(nfb);
    CdefList  dlist[MI_SIZE_128X128 * MI_SIZE_128X128];
    DECLARE_ALIGNED(32, uint16_t, inbuf[CDEF_INBUF_SIZE]);
    uint16_t *in = inbuf + CDEF_VBORDER * CDEF_BSTRIDE + CDEF_HBORDER;
    DECLARE_ALIGNED(32, uint16_t, tmp_dst[1 << (MAX_SB_SIZE_LOG2 * 2)]);
    const int pri_damping = 3 + (q >> 6);
    static const int bsz[3] = {BLOCK_8X8, BLOCK_4X4, BLOCK_4X4};
    for (int fbr = 0; fbr < nvfb && (g_stages & 2); fbr++)
        for (int fbc = 0; fbc < nhfb; fbc++) {
            const int fb = fbr * nhfb + fbc, lr = 16 * fbr, lc = 16 * fbc;
            const int nhb = AOMMIN(16, mi_cols - lc), nvb = AOMMIN(16, mi_rows - lr);
            int       dirinit = 0;
            uint8_t   dir[CDEF_NBLOCKS][CDEF_NBLOCKS];
            int32_t   var[CDEF_NBLOCKS][CDEF_NBLOCKS];
            const int cnt = svt_sb_compute_cdef_list(pcs, cm, lr, lc, dlist, BLOCK_64X64);
            skipfb[fb]    = cnt == 0;
            if (!cnt) continue;
            for (int pli = 0; pli < 3; pli++) {
                const int sub = pli > 0, mi_l2 = 2 - sub, pw = W >> sub;
                if (pli < 2) memset(inbuf, (uint8_t)CDEF_VERY_LARGE, sizeof inbuf);
                const int yoff = CDEF_VBORDER * (fbr != 0), xoff = CDEF_HBORDER * (fbc != 0);
                const int ysize = (nvb << mi_l2) + CDEF_VBORDER * (fbr + 1 < nvfb) + yoff;
                const int xsize = (nhb << mi_l2) + CDEF_HBORDER * (fbc + 1 < nhfb) + xoff;
                svt_aom_copy_sb8_16(&in[-yoff * CDEF_BSTRIDE - xoff], CDEF_BSTRIDE,
                                    is16 ? (uint8_t *)rec[pli] : rec8[pli], (lr << mi_l2) - yoff, (lc << mi_l2) - xoff,
                                    pw, ysize, xsize, is16);
                const uint8_t ssf = AOMMIN(cctl.subsampling_factor, pli ? 1 : 4);
                for (int gi = 0; gi < nstr; gi++) {
                    const int first = gi < cctl.first_pass_fs_num;
                    const int k     = first ? gi : gi - cctl.first_pass_fs_num;
                    if (pli && (first ? cctl.default_first_pass_fs_uv[k] : cctl.default_second_pass_fs_uv[k]) == -1) {
                        mse[nfb + fb][gi] = 1040400ull * 64;
                        continue;
                    }
                    const int fs = first ? cctl.default_first_pass_fs[k] : cctl.default_second_pass_fs[k];
                    const int ps = fs / CDEF_SEC_STRENGTHS, ss = fs % CDEF_SEC_STRENGTHS;
                    svt_cdef_filter_fb(is16 ? NULL : (uint8_t *)tmp_dst, is16 ? tmp_dst : NULL, 0, in, sub, sub, dir,
                                       &dirinit, var, pli, dlist, cnt, ps, ss + (ss == 3), pri_damping, pri_damping,
                                       cs, ssf);
                    const size_t   o = (size_t)(lr << mi_l2) * pw + (lc << mi_l2);
                    const uint64_t d =
                        is16 ? svt_compute_cdef_dist_16bit(src[pli] + o, pw, tmp_dst, dlist, cnt, (BlockSize)bsz[pli], cs,
                                                           pli, ssf)
                             : svt_compute_cdef_dist_8bit(src8[pli] + o, pw, (uint8_t *)tmp_dst, dlist, cnt,
                                                          (BlockSize)bsz[pli], cs, pli, ssf);
                    if (pli < 2)
                        mse[pli * nfb + fb][gi] = d * ssf;
                    else
                        mse[nfb + fb][gi] += d * ssf;
                }
            }
        }
    ts[2] = now();
    /* ---- CDEF pick: finish_cdef_search's greedy + RD (EbEncCdef.c:697-890) ---- */
    uint64_t **m0 = xmalloc(sizeof(uint64_t *) * nfb), **m1 = xmalloc(sizeof(uint64_t *) * nfb);
    int       *fbl = xmalloc(sizeof(int) * nfb), sb_count = 0;
    for (int fb = 0; fb < nfb && (g_stages & 2); fb++)
        if (!skipfb[fb]) {
            if (cctl.zero_fs_cost_bias)
                for (int p = 0; p < 2; p++) mse[p * nfb + fb][0] = (cctl.zero_fs_cost_bias * mse[p * nfb + fb][0]) >> 6;
            m0[sb_count] = mse[fb], m1[sb_count] = mse[nfb + fb], fbl[sb_count++] = fb;
        }
    uint64_t **mm[2] = {m0, m1};
    int        best_lev[4][2][16], nbits = 0;
    uint64_t   best_cost = (uint64_t)1 << 63;
    for (int i = 0; i <= 3 && (g_stages & 2); i++) {
        const int nb = 1 << i;
        int      *l0 = best_lev[i][0], *l1 = best_lev[i][1];
        memset(l0, 0, sizeof best_lev[i][0]), memset(l1, 0, sizeof best_lev[i][1]);
        uint64_t  tot = 0;
        for (int k = 0; k < nb; k++) tot = svt_search_one_dual(l0, l1, k, mm, sb_count, 0, nstr);
        for (int k = 0; k < 4 * nb; k++) {
            for (int j = 0; j < nb - 1; j++) l0[j] = l0[j + 1], l1[j] = l1[j + 1];
            tot = svt_search_one_dual(l0, l1, nb - 1, mm, sb_count, 0, nstr);
        }
        const int64_t  rate = (int64_t)(sb_count * i + nb * 6 * 2) << 9;
        const uint64_t cost = (uint64_t)(((rate * hdr[H_LAMBDA] + 256) >> 9) + ((int64_t)(tot * 16) << 7));
        if (cost < best_cost) best_cost = cost, nbits = i;
    }
    /* ---- CDEF apply: every listed 8x8 of every FB filtered with its strength, neighbours unfiltered ---- */
    for (int p = 0; p < 3; p++) {
        const size_t n = (size_t)(W >> (p > 0)) * (H >> (p > 0));
        cdf[p]         = xmalloc(2 * n);
        memcpy(cdf[p], rec[p], 2 * n);
    }
    const int nb = 1 << nbits;
    for (int s = 0; s < sb_count; s++) {
        const int fb = fbl[s], fbr = fb / nhfb, fbc = fb % nhfb, lr = 16 * fbr, lc = 16 * fbc;
        uint64_t  be = (uint64_t)1 << 63;
        int       bg = 0;
        for (int g = 0; g < nb; g++) {
            const uint64_t e = m0[s][best_lev[nbits][0][g]] + m1[s][best_lev[nbits][1][g]];
            if (e < be) be = e, bg = g;
        }
        const int gy = best_lev[nbits][0][bg], gu = best_lev[nbits][1][bg];
        const int nf = cctl.first_pass_fs_num;
        const int ys = gy < nf ? cctl.default_first_pass_fs[gy] : cctl.default_second_pass_fs[gy - nf];
        const int us = gu < nf ? cctl.default_first_pass_fs[gu] : cctl.default_second_pass_fs[gu - nf];
        int       lvl[3] = {ys / 4, us / 4, us / 4}, sec[3] = {ys % 4, us % 4, us % 4};
        for (int p = 0; p < 3; p++) sec[p] += sec[p] == 3;
        if (!lvl[0] && !sec[0] && !lvl[1] && !sec[1]) continue;
        const int nhb = AOMMIN(16, mi_cols - lc), nvb = AOMMIN(16, mi_rows - lr);
        const int cnt = svt_sb_compute_cdef_list(pcs, cm, lr, lc, dlist, BLOCK_64X64);
        int       dirinit = 0;
        uint8_t   dir[CDEF_NBLOCKS][CDEF_NBLOCKS];
        int32_t   var[CDEF_NBLOCKS][CDEF_NBLOCKS];
        for (int pli = 0; pli < 3; pli++) {
            if (!lvl[pli] && !sec[pli]) continue;
            const int sub = pli > 0, mi_l2 = 2 - sub, pw = W >> sub;
            memset(inbuf, (uint8_t)CDEF_VERY_LARGE, sizeof inbuf);
            const int yoff = CDEF_VBORDER * (fbr != 0), xoff = CDEF_HBORDER * (fbc != 0);
            const int ysize = (nvb << mi_l2) + CDEF_VBORDER * (fbr + 1 < nvfb) + yoff;
            const int xsize = (nhb << mi_l2) + CDEF_HBORDER * (fbc + 1 < nhfb) + xoff;
            svt_aom_copy_sb8_16(&in[-yoff * CDEF_BSTRIDE - xoff], CDEF_BSTRIDE,
                                is16 ? (uint8_t *)rec[pli] : rec8[pli], (lr << mi_l2) - yoff, (lc << mi_l2) - xoff, pw,
                                ysize, xsize, is16);
            const size_t o = (size_t)(lr << mi_l2) * pw + (lc << mi_l2);
            svt_cdef_filter_fb(is16 ? NULL : cdf8[pli] + o, is16 ? cdf[pli] + o : NULL, pw, in, sub, sub, dir, &dirinit,
                               var, pli, dlist, cnt, lvl[pli], sec[pli], pri_damping, pri_damping, cs, 1);
        }
    }
    ts[3] = now();
    /* ---- LR: whole-crop search (one segment) + RD finish + apply ---- */
    if (g_stages & 4) {
    cm->frm_size.frame_width = cm->frm_size.superres_upscaled_width = W;
    cm->frm_size.frame_height = cm->frm_size.superres_upscaled_height = H;
    cm->subsampling_x = cm->subsampling_y = 1, cm->use_highbitdepth = bd > 8, cm->bit_depth = bd;
    set_lr_ctrls(cm);
    x->rdmult = hdr[H_RDMULT];
    for (int k = 0; k < 3; k++) x->switchable_restore_cost[k] = hdr[H_SW0 + k];
    for (int k = 0; k < 2; k++) x->wiener_restore_cost[k] = hdr[H_WN0 + k], x->sgrproj_restore_cost[k] = hdr[H_SG0 + k];
    const int usize[3] = {256, 128, 128};
    for (int p = 0; p < 3; p++) pcs->rst_info[p].restoration_unit_size = usize[p];
    svt_av1_alloc_restoration_buffers(pcs, cm);
    for (int p = 0; p < 3; p++)
        pcs->rusi_picture[p] = xmalloc(sizeof(RestUnitSearchInfo) * pcs->rst_info[p].units_per_tile);
    pcs->rest_search_mutex          = svt_create_mutex();
    pcs->rest_segments_column_count = 1;
    pcs->rest_segments_row_count    = 1;
    Yv12BufferConfig yd, yc, ys, yt;
    memset(&yd, 0, sizeof yd), memset(&yc, 0, sizeof yc), memset(&ys, 0, sizeof ys), memset(&yt, 0, sizeof yt);
    svt_aom_realloc_frame_buffer(&yd, W, H, 1, 1, 1, 32, 0, NULL, NULL, NULL);
    svt_aom_realloc_frame_buffer(&yc, W, H, 1, 1, 1, 32, 0, NULL, NULL, NULL);
    svt_aom_realloc_frame_buffer(&ys, W, H, 1, 1, 1, 32, 0, NULL, NULL, NULL);
    svt_aom_realloc_frame_buffer(&yt, W, H, 1, 1, 1, 32, 0, NULL, NULL, NULL);
    to_y12(&yd, rec, W, H);
    to_y12(&yc, cdf, W, H);
    to_y12(&ys, src, W, H);
    svt_av1_loop_restoration_save_boundary_lines(&yd, cm, 0);
    svt_av1_loop_restoration_save_boundary_lines(&yc, cm, 1);
    cm->frame_to_show = &yc;
    restoration_seg_search(tmpbuf, &yc, &ys, &yt, pcs, 0);
    rest_finish_search(pcs);
    svt_av1_loop_restoration_filter_frame(tmpbuf, &yc, cm, 0);
    free(yd.buffer_alloc), free(yc.buffer_alloc), free(ys.buffer_alloc), free(yt.buffer_alloc);
    }
    ts[4] = now();
    if (g_verbose) {
        int nt[3][4] = {{0}};
        for (int p = 0; p < 3; p++)
            for (int u = 0; u < pcs->rst_info[p].units_per_tile; u++)
                nt[p][pcs->rst_info[p].unit_info[u].restoration_type & 3]++;
        fprintf(stderr,
                "crop %d,%d: dlf %d/%d/%d/%d cdef sb %d nbits %d  lr frame types %d %d %d, Y unit types %d %d %d %d\n",
                c->x0, c->y0, lf->filter_level[0], lf->filter_level[1], lf->filter_level_u, lf->filter_level_v,
                sb_count, nbits, pcs->rst_info[0].frame_restoration_type, pcs->rst_info[1].frame_restoration_type,
                pcs->rst_info[2].frame_restoration_type, nt[0][0], nt[0][1], nt[0][2], nt[0][3]);
    }
    /* ---- MD batch: every block shape <= 64x64 of every SB against every reference at its MV ---- */
    static const int sw[19] = {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 4, 16, 8, 32, 16, 64};
    static const int sh[19] = {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 16, 4, 32, 8, 64, 16};
    const int        nref = hdr[H_NREF], Wf = hdr[H_W], Hf = hdr[H_H], nsbx = (Wf + 63) / 64;
    volatile uint64_t sink = 0;
    for (int sy = 0; sy < H && (g_stages & 8); sy += 64)
        for (int sx = 0; sx < W; sx += 64) {
            const int sb = ((c->y0 + sy) / 64) * nsbx + (c->x0 + sx) / 64;
            uint16_t *s  = g_src[0] + (size_t)(c->y0 + sy) * Wf + c->x0 + sx;
            for (int r = 0; r < nref; r++) {
                int ry = c->y0 + sy + g_mv[((size_t)sb * nref + r) * 2 + 1], rx = c->x0 + sx + g_mv[((size_t)sb * nref + r) * 2];
                ry = ry < 0 ? 0 : ry > Hf - 64 ? Hf - 64 : ry; /* whole block inside the reference */
                rx = rx < 0 ? 0 : rx > Wf - 64 ? Wf - 64 : rx;
                uint16_t *rf = g_ref[r] + (size_t)ry * Wf + rx;
                for (int k = 0; k < 19; k++)
                    for (int by = 0; by < 64; by += sh[k])
                        for (int bx = 0; bx < 64; bx += sw[k]) {
                            uint16_t *a = s + (size_t)by * Wf + bx, *b = rf + (size_t)by * Wf + bx;
                            uint32_t  sse;
                            sink += svt_aom_sad_16bit_kernel_avx2(a, Wf, b, Wf, sh[k], sw[k]);
                            sink += (uint64_t)svt_aom_highbd_sse_avx2((uint8_t *)a, Wf, (uint8_t *)b, Wf, sw[k],
                                                                      sh[k]);
                            sink += svt_aom_variance_highbd_c(a, Wf, b, Wf, sw[k], sh[k], &sse);
                        }
            }
        }
    (void)sink;
    ts[5] = now();
    pthread_mutex_lock(&g_stage_lock);
    for (int k = 0; k < 5; k++) g_stage[k] += ts[k + 1] - ts[k];
    pthread_mutex_unlock(&g_stage_lock);
    /* buffers of the crop (the picture structures' own allocations are left to process exit) */
    for (int p = 0; p < 3; p++) free(src[p]), free(rec[p]), free(trl[p]), free(cdf[p]);
    free(mse), free(skipfb), free(m0), free(m1), free(fbl), free(blocks), free(cells);
    for (int p = 0; p < 3; p++) free(src8[p]), free(rec8[p]), free(cdf8[p]);
}

/* ------------------------------------------------------------------------------------------- threads */
static Crop           *g_jobs;
static int             g_njobs, g_next;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static void *worker(void *arg) {
    (void)arg;
    int32_t *tmpbuf = xmalloc(RESTORATION_TMPBUF_SIZE);
    for (;;) {
        pthread_mutex_lock(&g_lock);
        const int j = g_next < g_njobs ? g_next++ : -1;
        pthread_mutex_unlock(&g_lock);
        if (j < 0) break;
        run_crop(&g_jobs[j], tmpbuf);
    }
    free(tmpbuf);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <input.bin> <threads>\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 1;
    }
    read_all(f, hdr, sizeof hdr);
    read_all(f, &cctl, sizeof cctl);
    const int W = hdr[H_W], H = hdr[H_H], nref = hdr[H_NREF];
    if (getenv("REF_BENCH_STAGES")) g_stages = atoi(getenv("REF_BENCH_STAGES")) & 15;
    if ((hdr[H_BD] != 10 && !(hdr[H_BD] == 8 && g_stages == 2)) || (W & 63) || (H & 7) || nref < 0 || nref > 16) {
        fprintf(stderr, "ref_bench: unsupported input (10-bit, or 8-bit with the CDEF stage alone; width multiple of 64)\n");
        return 1;
    }
    for (int k = 0; k < 2; k++) {
        uint16_t **pl = k ? g_rec : g_src;
        for (int p = 0; p < 3; p++) {
            const size_t n = (size_t)(W >> (p > 0)) * (H >> (p > 0));
            pl[p]          = xmalloc(2 * n);
            read_all(f, pl[p], 2 * n);
        }
    }
    g_mi = xmalloc(sizeof(SvtGpuLfMi) * (size_t)(H >> 2) * (W >> 2));
    read_all(f, g_mi, sizeof(SvtGpuLfMi) * (size_t)(H >> 2) * (W >> 2));
    g_ref = xmalloc(sizeof(uint16_t *) * (nref ? nref : 1));
    for (int r = 0; r < nref; r++) {
        g_ref[r] = xmalloc(2 * (size_t)W * H);
        read_all(f, g_ref[r], 2 * (size_t)W * H);
    }
    const size_t nsb = (size_t)((W + 63) / 64) * ((H + 63) / 64);
    g_mv             = xmalloc(sizeof(int32_t) * nsb * (nref ? nref : 1) * 2);
    read_all(f, g_mv, sizeof(int32_t) * nsb * nref * 2);
    fclose(f);
    bind_kernels();
    g_verbose = getenv("REF_BENCH_VERBOSE") != NULL;
    const int gx = hdr[H_GX], gy = hdr[H_GY], cw = (W / gx) & ~63, ch = (H / gy) & ~63;
    const int passes = argc > 3 && atoi(argv[3]) > 0 ? atoi(argv[3]) : 1;
    g_njobs          = gx * gy * passes;
    g_jobs           = xmalloc(sizeof(Crop) * g_njobs);
    for (int j = 0; j < g_njobs; j++) g_jobs[j] = (Crop){cw, ch, (j % gx) * cw, (j / gx % gy) * ch};
    int nthr = atoi(argv[2]);
    if (nthr < 1) nthr = 1;
    if (nthr > gx * gy) nthr = gx * gy;
    pthread_t      th[64];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthr && t < 64; t++) pthread_create(&th[t], NULL, worker, NULL);
    for (int t = 0; t < nthr && t < 64; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double dt = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("ref_bench px=%lld seconds=%.4f threads=%d\n", (long long)g_njobs * cw * ch, dt, nthr);
    fprintf(stderr, "thread-seconds: dlf %.3f cdef_search %.3f cdef_pick_apply %.3f lr %.3f md %.3f\n", g_stage[0],
            g_stage[1], g_stage[2], g_stage[3], g_stage[4]);
    return 0;
}
