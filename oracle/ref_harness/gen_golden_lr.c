/*
 * gen_golden_lr.c — loop-restoration golden vectors (test infrastructure; never shipped).
 *
 * Links the REFERENCE's own C (convolve.c, EbRestoration.c, EbPictureBufferDesc.c, EbPictureOperators.c, compiled
 * from /root/reference by oracle/ref.mk) and records on deterministic SplitMix64 inputs:
 *   lr_wiener.bin  svt_av1_(highbd_)wiener_convolve_add_src_c, bd 8/10/12, legal random taps
 *   lr_sgr.bin     svt_av1_selfguided_restoration_c (flt0/flt1, all 16 eps) and svt_apply_selfguided_restoration_c
 *   lr_frame.bin   svt_av1_loop_restoration_filter_frame on whole frames with stripe boundary lines saved by
 *                  svt_av1_loop_restoration_save_boundary_lines from a deblocked frame and a CDEF frame
 * usage: gen_golden_lr <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbRestoration.h"
#include "EbPictureControlSet.h"
#include "Av1Common.h"
#include "common_dsp_rtcd.h"
#include "aom_dsp_rtcd.h"
#include "EbCodingUnit.h"
#include "EbThreads.h"
#include "golden_io.h"

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

static void bind_c_kernels(void) {
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

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* legal Wiener taps (AV1: taps 0..2 in [-5,10], [-23,8], [-17,46]; centre = -2 * sum; tap 7 = 0) */
static void rand_wiener(Rng *r, int16_t *f, int chroma) {
    static const int lo[3] = {-5, -23, -17}, hi[3] = {10, 8, 46};
    int              t[3];
    for (int k = 0; k < 3; k++) t[k] = lo[k] + (int)rng_below(r, (uint32_t)(hi[k] - lo[k] + 1));
    if (chroma) t[0] = 0;
    f[0] = f[6] = (int16_t)t[0];
    f[1] = f[5] = (int16_t)t[1];
    f[2] = f[4] = (int16_t)t[2];
    f[3]        = (int16_t)(-2 * (t[0] + t[1] + t[2]));
    f[7]        = 0;
}

static int rand_px(Rng *r, int bd, int base, int kind) {
    const int maxv = (1 << bd) - 1;
    int       v;
    if (kind == 0)
        v = (int)rng_below(r, (uint32_t)maxv + 1);
    else
        v = base + (int)rng_below(r, (uint32_t)(1 << (bd - 5))) - (1 << (bd - 6));
    return clampi(v, 0, maxv);
}

/* ------------------------------------------------------------------------------------------- */
#define WN 120
static void gen_wiener(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/lr_wiener.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4C52000000000001ull};
    /* per case: meta {bd, w, h}, taps fx[8], fy[8], input (h+8) x (w+8) from (-3,-3), output h x w */
    const int IS = 72 * 72, OS = 64 * 64;
    int32_t  *meta = calloc(WN, 3 * sizeof(int32_t));
    int16_t  *taps = calloc(WN, 16 * sizeof(int16_t));
    uint16_t *in   = calloc(WN, IS * sizeof(uint16_t));
    uint16_t *out  = calloc(WN, OS * sizeof(uint16_t));
    static const int ws[5] = {16, 32, 48, 64, 8};
    for (int n = 0; n < WN; n++) {
        const int bd = n < 40 ? 8 : n < 80 ? 10 : 12;
        const int w = ws[rng_below(&r, 5)], h = 1 + (int)rng_below(&r, 64);
        const int st = w + 8, base = (int)rng_below(&r, 1u << bd), kind = (int)rng_below(&r, 2);
        DECLARE_ALIGNED(16, int16_t, fx[8]);
        DECLARE_ALIGNED(16, int16_t, fy[8]);
        rand_wiener(&r, fx, n % 3 == 2);
        rand_wiener(&r, fy, n % 3 == 2);
        uint16_t *I = in + (size_t)n * IS, *O = out + (size_t)n * OS;
        for (int k = 0; k < (h + 8) * st; k++) I[k] = (uint16_t)rand_px(&r, bd, base, kind);
        ConvolveParams cp;
        memset(&cp, 0, sizeof cp);
        cp.round_0 = 3;
        cp.round_1 = 11;
        if (bd + 7 - 3 + 2 > 16) {
            cp.round_0 += bd + 7 - 3 + 2 - 16;
            cp.round_1 -= bd + 7 - 3 + 2 - 16;
        }
        if (bd == 8) {
            uint8_t *i8 = malloc((size_t)(h + 8) * st), *o8 = malloc((size_t)h * w);
            for (int k = 0; k < (h + 8) * st; k++) i8[k] = (uint8_t)I[k];
            svt_av1_wiener_convolve_add_src_c(i8 + 3 * st + 3, st, o8, w, fx, fy, w, h, &cp);
            for (int k = 0; k < h * w; k++) O[k] = o8[k];
            free(i8);
            free(o8);
        } else {
            svt_av1_highbd_wiener_convolve_add_src_c(CONVERT_TO_BYTEPTR(I + 3 * st + 3), st, CONVERT_TO_BYTEPTR(O), w, fx,
                                                     fy, w, h, &cp, bd);
        }
        meta[3 * n] = bd, meta[3 * n + 1] = w, meta[3 * n + 2] = h;
        memcpy(taps + 16 * n, fx, 16);
        memcpy(taps + 16 * n + 8, fy, 16);
        char nm[32];
        snprintf(nm, sizeof nm, "in%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)(h + 8), (uint32_t)st, I);
        snprintf(nm, sizeof nm, "out%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)h, (uint32_t)w, O);
    }
    golden_put2(&g, "meta", 'i', WN, 3, meta);
    golden_put2(&g, "taps", 'h', WN, 16, taps);
    golden_close(&g);
    free(meta), free(taps), free(in), free(out);
}

/* ------------------------------------------------------------------------------------------- */
#define SN 48
static void gen_sgr(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/lr_sgr.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4C52000000000002ull};
    /* per case: meta {bd, w, h, eps, xqd0, xqd1}, input (h+6) x (w+6) from (-3,-3), flt0/flt1/out h x w */
    const int IS = 70 * 70, OS = 64 * 64;
    int32_t  *meta = calloc(SN, 6 * sizeof(int32_t));
    uint16_t *in   = calloc(SN, IS * sizeof(uint16_t));
    int32_t  *f0   = calloc(SN, OS * sizeof(int32_t)), *f1 = calloc(SN, OS * sizeof(int32_t));
    uint16_t *out  = calloc(SN, OS * sizeof(uint16_t));
    int32_t  *tmp  = malloc(RESTORATION_UNITPELS_MAX * 2 * sizeof(int32_t));
    for (int n = 0; n < SN; n++) {
        const int bd = n & 1 ? 10 : 8, eps = (n * 5) & 15;
        const int w = 8 + (int)rng_below(&r, 57), h = 8 + (int)rng_below(&r, 57);
        const int st = w + 6, base = (int)rng_below(&r, 1u << bd), kind = (int)rng_below(&r, 3) != 0;
        uint16_t *I = in + (size_t)n * IS;
        for (int k = 0; k < (h + 6) * st; k++) I[k] = (uint16_t)rand_px(&r, bd, base, kind);
        const int32_t xqd[2] = {-96 + (int)rng_below(&r, 128), -32 + (int)rng_below(&r, 128)};
        uint8_t      *i8     = malloc((size_t)(h + 6) * st);
        for (int k = 0; k < (h + 6) * st; k++) i8[k] = (uint8_t)I[k];
        const uint8_t *src = bd > 8 ? CONVERT_TO_BYTEPTR(I + 3 * st + 3) : i8 + 3 * st + 3;
        svt_av1_selfguided_restoration_c(src, w, h, st, f0 + (size_t)n * OS, f1 + (size_t)n * OS, w, eps, bd, bd > 8);
        uint16_t *O = out + (size_t)n * OS;
        if (bd > 8)
            svt_apply_selfguided_restoration_c(src, w, h, st, eps, xqd, CONVERT_TO_BYTEPTR(O), w, tmp, bd, 1);
        else {
            uint8_t *o8 = malloc((size_t)w * h);
            svt_apply_selfguided_restoration_c(src, w, h, st, eps, xqd, o8, w, tmp, bd, 0);
            for (int k = 0; k < w * h; k++) O[k] = o8[k];
            free(o8);
        }
        free(i8);
        int32_t *m = meta + 6 * n;
        m[0] = bd, m[1] = w, m[2] = h, m[3] = eps, m[4] = xqd[0], m[5] = xqd[1];
        char nm[32];
        snprintf(nm, sizeof nm, "in%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)(h + 6), (uint32_t)st, I);
        snprintf(nm, sizeof nm, "flt0_%d", n);
        golden_put2(&g, nm, 'i', (uint32_t)h, (uint32_t)w, f0 + (size_t)n * OS);
        snprintf(nm, sizeof nm, "flt1_%d", n);
        golden_put2(&g, nm, 'i', (uint32_t)h, (uint32_t)w, f1 + (size_t)n * OS);
        snprintf(nm, sizeof nm, "out%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)h, (uint32_t)w, O);
    }
    golden_put2(&g, "meta", 'i', SN, 6, meta);
    golden_close(&g);
    free(meta), free(in), free(f0), free(f1), free(out), free(tmp);
}

/* ------------------------------------------------------------------------------------------- */
typedef struct LrCase {
    int w, h, bd, usize, types[3];
} LrCase;

static void fill_frame(Yv12BufferConfig *f, int bd, Rng *r, const Yv12BufferConfig *like, int noise) {
    for (int p = 0; p < 3; p++) {
        const int pw = f->crop_widths[p > 0], ph = f->crop_heights[p > 0], st = f->strides[p > 0];
        const int maxv = (1 << bd) - 1;
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) {
                int v;
                if (like) {
                    const int o = bd > 8 ? CONVERT_TO_SHORTPTR(like->buffers[p])[y * st + x] : like->buffers[p][y * st + x];
                    v           = o + (int)rng_below(r, 2 * noise + 1) - noise;
                } else
                    v = (x * 3 + y * 2) * (maxv + 1) / 1024 + (int)rng_below(r, (uint32_t)(maxv / 8 + 1)) +
                        ((x / 8 + y / 8) & 1) * (maxv / 16);
                v = clampi(v, 0, maxv);
                if (bd > 8)
                    CONVERT_TO_SHORTPTR(f->buffers[p])[y * st + x] = (uint16_t)v;
                else
                    f->buffers[p][y * st + x] = (uint8_t)v;
            }
    }
}

static void put_frame(GoldenFile *g, const char *tag, int ci, const Yv12BufferConfig *f, int bd) {
    for (int p = 0; p < 3; p++) {
        const int pw = f->crop_widths[p > 0], ph = f->crop_heights[p > 0], st = f->strides[p > 0];
        uint16_t *a  = malloc(sizeof(uint16_t) * pw * ph);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++)
                a[y * pw + x] = bd > 8 ? CONVERT_TO_SHORTPTR(f->buffers[p])[y * st + x] : f->buffers[p][y * st + x];
        char nm[64];
        snprintf(nm, sizeof nm, "c%d_%s%d", ci, tag, p);
        golden_put2(g, nm, 'H', (uint32_t)ph, (uint32_t)pw, a);
        free(a);
    }
}

static void gen_frames(const char *dir) {
    static const LrCase cases[] = {
        {200, 136, 8, 64, {3, 1, 2}},   {256, 200, 10, 64, {3, 3, 3}}, {136, 72, 10, 128, {1, 0, 2}},
        {320, 256, 8, 128, {2, 1, 0}},  {392, 232, 10, 256, {3, 3, 1}}, {64, 48, 8, 64, {3, 2, 2}},
        /* crop sizes that are not multiples of 8 (frm_size.frame_width = input width - pad): odd chroma widths and
         * heights, a last unit column and stripe ending inside a 4-sample group */
        {202, 138, 10, 64, {3, 3, 3}},  {134, 74, 8, 64, {1, 2, 3}},   {250, 90, 10, 128, {2, 3, 1}},
    };
    const int ncase = (int)(sizeof(cases) / sizeof(cases[0]));
    char      path[512];
    snprintf(path, sizeof path, "%s/lr_frame.bin", dir);
    GoldenFile g  = golden_open(path);
    Rng        r  = {0x4C52000000000003ull};
    uint32_t   nc = (uint32_t)ncase;
    golden_put1(&g, "ncase", 'I', 1, &nc);
    int32_t *tmpbuf = malloc(RESTORATION_TMPBUF_SIZE);
    for (int ci = 0; ci < ncase; ci++) {
        const LrCase *c = &cases[ci];
        const int     hb = c->bd > 8;
        Av1Common    *cm = calloc(1, sizeof(Av1Common));
        PictureControlSet *pcs = calloc(1, sizeof(PictureControlSet));
        cm->child_pcs                    = pcs;
        cm->frm_size.frame_width         = c->w;
        cm->frm_size.frame_height        = c->h;
        cm->frm_size.superres_upscaled_width  = c->w;
        cm->frm_size.superres_upscaled_height = c->h;
        cm->subsampling_x = cm->subsampling_y = 1;
        cm->use_highbitdepth             = hb;
        cm->bit_depth                    = c->bd;
        cm->mi_rows                      = ((c->h + 7) & ~7) >> 2;
        cm->mi_cols                      = ((c->w + 7) & ~7) >> 2;
        int usize[3]                     = {c->usize, c->usize >> 1, c->usize >> 1};
        for (int p = 0; p < 3; p++) pcs->rst_info[p].restoration_unit_size = usize[p];
        svt_av1_alloc_restoration_buffers(pcs, cm);
        Yv12BufferConfig dlf, cdef;
        memset(&dlf, 0, sizeof dlf);
        memset(&cdef, 0, sizeof cdef);
        svt_aom_realloc_frame_buffer(&dlf, c->w, c->h, 1, 1, hb, 32, 0, NULL, NULL, NULL);
        svt_aom_realloc_frame_buffer(&cdef, c->w, c->h, 1, 1, hb, 32, 0, NULL, NULL, NULL);
        fill_frame(&dlf, c->bd, &r, NULL, 0);
        fill_frame(&cdef, c->bd, &r, &dlf, 3 << (c->bd - 8));
        put_frame(&g, "dlf", ci, &dlf, c->bd);
        put_frame(&g, "cdef", ci, &cdef, c->bd);
        svt_av1_loop_restoration_save_boundary_lines(&dlf, cm, 0);
        svt_av1_loop_restoration_save_boundary_lines(&cdef, cm, 1);
        /* unit parameters: {type, vfilter[8], hfilter[8], ep, xqd0, xqd1} per unit */
        char    nm[64];
        int32_t prm[6] = {c->w, c->h, c->bd, c->usize, 0, 0};
        for (int p = 0; p < 3; p++) {
            RestorationInfo *rsi = &pcs->rst_info[p];
            rsi->frame_restoration_type = c->types[p] == 0 ? RESTORE_NONE : RESTORE_SWITCHABLE;
            const int nu = rsi->units_per_tile;
            int32_t  *u  = calloc((size_t)nu, 20 * sizeof(int32_t));
            for (int k = 0; k < nu; k++) {
                RestorationUnitInfo *ui = &rsi->unit_info[k];
                memset(ui, 0, sizeof *ui);
                int t = c->types[p] == 3 ? (int)rng_below(&r, 3) : c->types[p];
                if (c->types[p] == 0) t = 0;
                ui->restoration_type = (RestorationType)t;
                rand_wiener(&r, ui->wiener_info.vfilter, p > 0);
                rand_wiener(&r, ui->wiener_info.hfilter, p > 0);
                ui->sgrproj_info.ep     = (int)rng_below(&r, 16);
                ui->sgrproj_info.xqd[0] = -96 + (int)rng_below(&r, 128);
                ui->sgrproj_info.xqd[1] = -32 + (int)rng_below(&r, 128);
                int32_t *e = u + 20 * k;
                e[0]       = t;
                for (int q = 0; q < 8; q++) e[1 + q] = ui->wiener_info.vfilter[q], e[9 + q] = ui->wiener_info.hfilter[q];
                e[17] = ui->sgrproj_info.ep, e[18] = ui->sgrproj_info.xqd[0], e[19] = ui->sgrproj_info.xqd[1];
            }
            snprintf(nm, sizeof nm, "c%d_units%d", ci, p);
            golden_put2(&g, nm, 'i', (uint32_t)nu, 20, u);
            free(u);
            prm[4] |= (c->types[p] != 0) << p;
        }
        snprintf(nm, sizeof nm, "c%d_params", ci);
        golden_put1(&g, nm, 'i', 6, prm);
        svt_av1_loop_restoration_filter_frame(tmpbuf, &cdef, cm, 0);
        put_frame(&g, "out", ci, &cdef, c->bd);
        free(dlf.buffer_alloc);
        free(cdef.buffer_alloc);
    }
    free(tmpbuf);
    golden_close(&g);
}

/* ------------------------------------------------------------------------------------------- */
/* whole-frame search: restoration_seg_search (one segment) + rest_finish_search                  */
/* ------------------------------------------------------------------------------------------- */
typedef struct SearchCase {
    int w, h, bd, usize, wn, sg;
} SearchCase;

static void set_ctrls(Av1Common *cm, int wn, int sg) {
    WnFilterCtrls *w = &cm->wn_filter_ctrls;
    SgFilterCtrls *g = &cm->sg_filter_ctrls;
    memset(w, 0, sizeof *w);
    memset(g, 0, sizeof *g);
    /* svt_aom_set_wn_filter_ctrls / svt_aom_set_sg_filter_ctrls (EncModeConfig.c:1329-1445) are static: the
     * same values are written here */
    if (wn) {
        w->enabled = 1, w->use_chroma = wn <= 4, w->filter_tap_lvl = wn <= 2 ? 1 : 2;
        w->use_refinement = wn <= 3, w->max_one_refinement_step = wn >= 2, w->use_prev_frame_coeffs = 0;
    }
    if (sg) {
        g->enabled = 1, g->use_chroma = sg <= 3, g->step_range = 16;
        g->start_ep[0] = 0, g->end_ep[0] = 16, g->ep_inc[0] = sg >= 3 ? 8 : 1;
        g->start_ep[1] = sg == 1 ? 0 : 4, g->end_ep[1] = sg == 1 ? 16 : 5, g->ep_inc[1] = 1;
        g->refine[0] = 1, g->refine[1] = sg == 1;
    }
}

static void gen_search(const char *dir) {
    static const SearchCase cases[] = {
        {136, 72, 8, 64, 1, 1}, {200, 136, 10, 64, 1, 1}, {256, 144, 10, 128, 2, 2},
        {160, 96, 8, 64, 3, 3}, {128, 128, 10, 64, 4, 4}, {96, 64, 8, 128, 1, 0},
        /* crop sizes that are not multiples of 8 (see gen_frames) */
        {202, 138, 10, 64, 1, 1}, {134, 74, 8, 64, 2, 2}, {250, 90, 10, 128, 1, 1}, {198, 102, 8, 64, 3, 3},
        /* one restoration type searched for luma only (Wiener level 5 of presets 3-9 beside self-guided level 3 / 1,
         * self-guided level 4 beside Wiener level 1): rest_finish_search's switchable pass over a chroma plane then
         * reads the luma plane's entries of the shared rusi array for the type chroma did not search */
        {264, 200, 10, 64, 5, 3}, {200, 136, 8, 64, 5, 1}, {192, 128, 10, 64, 1, 4}, {328, 184, 10, 64, 5, 3},
    };
    const int ncase = (int)(sizeof(cases) / sizeof(cases[0]));
    char      path[512];
    snprintf(path, sizeof path, "%s/lr_search.bin", dir);
    GoldenFile g  = golden_open(path);
    Rng        r  = {0x4C52000000000004ull};
    uint32_t   nc = (uint32_t)ncase;
    golden_put1(&g, "ncase", 'I', 1, &nc);
    int32_t *tmpbuf = malloc(RESTORATION_TMPBUF_SIZE);
    for (int ci = 0; ci < ncase; ci++) {
        const SearchCase *c  = &cases[ci];
        const int         hb = c->bd > 8;
        Av1Common               *cm   = calloc(1, sizeof(Av1Common));
        PictureControlSet       *pcs  = calloc(1, sizeof(PictureControlSet));
        PictureParentControlSet *ppcs = calloc(1, sizeof(PictureParentControlSet));
        Macroblock              *x    = calloc(1, sizeof(Macroblock));
        pcs->ppcs                     = ppcs;
        ppcs->av1_cm                  = cm;
        ppcs->av1x                    = x;
        cm->child_pcs                 = pcs;
        cm->frm_size.frame_width = cm->frm_size.superres_upscaled_width = c->w;
        cm->frm_size.frame_height = cm->frm_size.superres_upscaled_height = c->h;
        cm->subsampling_x = cm->subsampling_y = 1;
        cm->use_highbitdepth                   = hb;
        cm->bit_depth                          = c->bd;
        cm->mi_rows                            = ((c->h + 7) & ~7) >> 2; /* the 8-aligned coded size */
        cm->mi_cols                            = ((c->w + 7) & ~7) >> 2;
        set_ctrls(cm, c->wn, c->sg);
        x->rdmult = 1000 + (int)rng_below(&r, 20000);
        for (int k = 0; k < 3; k++) x->switchable_restore_cost[k] = 100 + (int)rng_below(&r, 2000);
        for (int k = 0; k < 2; k++) x->wiener_restore_cost[k] = 100 + (int)rng_below(&r, 2000);
        for (int k = 0; k < 2; k++) x->sgrproj_restore_cost[k] = 100 + (int)rng_below(&r, 2000);
        const int usize[3] = {c->usize, c->usize >> 1, c->usize >> 1};
        for (int p = 0; p < 3; p++) pcs->rst_info[p].restoration_unit_size = usize[p];
        svt_av1_alloc_restoration_buffers(pcs, cm);
        for (int p = 0; p < 3; p++) pcs->rusi_picture[p] = calloc(pcs->rst_info[p].units_per_tile, sizeof(RestUnitSearchInfo));
        pcs->rest_search_mutex          = svt_create_mutex();
        pcs->rest_segments_column_count = 1;
        pcs->rest_segments_row_count    = 1;
        Yv12BufferConfig rec, src, trial;
        memset(&rec, 0, sizeof rec);
        memset(&src, 0, sizeof src);
        memset(&trial, 0, sizeof trial);
        svt_aom_realloc_frame_buffer(&rec, c->w, c->h, 1, 1, hb, 32, 0, NULL, NULL, NULL);
        svt_aom_realloc_frame_buffer(&src, c->w, c->h, 1, 1, hb, 32, 0, NULL, NULL, NULL);
        svt_aom_realloc_frame_buffer(&trial, c->w, c->h, 1, 1, hb, 32, 0, NULL, NULL, NULL);
        fill_frame(&src, c->bd, &r, NULL, 0);
        fill_frame(&rec, c->bd, &r, &src, 6 << (c->bd - 8));
        put_frame(&g, "src", ci, &src, c->bd);
        put_frame(&g, "rec", ci, &rec, c->bd);
        cm->frame_to_show = &rec; /* search_norestore_seg reads the unfiltered recon through it */
        restoration_seg_search(tmpbuf, &rec, &src, &trial, pcs, 0);
        rest_finish_search(pcs);
        char    nm[64];
        int32_t prm[16] = {c->w, c->h, c->bd, c->usize, c->wn, c->sg, x->rdmult, x->switchable_restore_cost[0],
                           x->switchable_restore_cost[1], x->switchable_restore_cost[2], x->wiener_restore_cost[0],
                           x->wiener_restore_cost[1], x->sgrproj_restore_cost[0], x->sgrproj_restore_cost[1], 0, 0};
        snprintf(nm, sizeof nm, "c%d_params", ci);
        golden_put1(&g, nm, 'i', 16, prm);
        int32_t ft[3];
        for (int p = 0; p < 3; p++) {
            const RestorationInfo *rsi = &pcs->rst_info[p];
            ft[p]                      = rsi->frame_restoration_type;
            const int nu               = rsi->units_per_tile;
            /* per unit: {type, vfilter[8], hfilter[8], ep, xqd0, xqd1} of the final unit info, and the search record
             * {sse none, sse wiener (or -1 = INT64_MAX), sse sgr, wiener v[8] h[8], sgr ep xqd0 xqd1} */
            int32_t *u  = calloc((size_t)nu, 20 * sizeof(int32_t));
            int64_t *ss = calloc((size_t)nu, 3 * sizeof(int64_t));
            int32_t *sp = calloc((size_t)nu, 19 * sizeof(int32_t));
            for (int k = 0; k < nu; k++) {
                const RestorationUnitInfo *ui = &rsi->unit_info[k];
                int32_t                   *e  = u + 20 * k;
                e[0]                          = ft[p] == RESTORE_NONE ? 0 : ui->restoration_type;
                /* only the parameters of the unit's own type: the reference leaves the others unwritten */
                if (e[0] == RESTORE_WIENER)
                    for (int q = 0; q < 8; q++) e[1 + q] = ui->wiener_info.vfilter[q], e[9 + q] = ui->wiener_info.hfilter[q];
                if (e[0] == RESTORE_SGRPROJ)
                    e[17] = ui->sgrproj_info.ep, e[18] = ui->sgrproj_info.xqd[0], e[19] = ui->sgrproj_info.xqd[1];
                const RestUnitSearchInfo *rs = &pcs->rusi_picture[p][k];
                for (int q = 0; q < 3; q++) ss[3 * k + q] = rs->sse[q] == INT64_MAX ? -1 : rs->sse[q];
                for (int q = 0; q < 8; q++) sp[19 * k + q] = rs->wiener.vfilter[q], sp[19 * k + 8 + q] = rs->wiener.hfilter[q];
                sp[19 * k + 16] = rs->sgrproj.ep, sp[19 * k + 17] = rs->sgrproj.xqd[0], sp[19 * k + 18] = rs->sgrproj.xqd[1];
            }
            snprintf(nm, sizeof nm, "c%d_units%d", ci, p);
            golden_put2(&g, nm, 'i', (uint32_t)nu, 20, u);
            snprintf(nm, sizeof nm, "c%d_sse%d", ci, p);
            golden_put2(&g, nm, 'q', (uint32_t)nu, 3, ss);
            snprintf(nm, sizeof nm, "c%d_rec%d_params", ci, p);
            golden_put2(&g, nm, 'i', (uint32_t)nu, 19, sp);
            free(u), free(ss), free(sp);
        }
        snprintf(nm, sizeof nm, "c%d_ftype", ci);
        golden_put1(&g, nm, 'i', 3, ft);
        free(rec.buffer_alloc), free(src.buffer_alloc), free(trial.buffer_alloc);
    }
    free(tmpbuf);
    golden_close(&g);
}

/* svt_av1_compute_stats(_highbd)_c on random units (win 7/5/3, bd 8/10/12) */
static void gen_stats(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/lr_stats.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4C52000000000005ull};
    const int  N = 18;
    int32_t    meta[18 * 6];
    for (int n = 0; n < N; n++) {
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12, win = n % 9 < 3 ? 7 : n % 9 < 6 ? 5 : 3;
        const int w = 16 + (int)rng_below(&r, 100), h = 16 + (int)rng_below(&r, 80), st = w + 8;
        uint16_t *d = malloc(sizeof(uint16_t) * st * (h + 8)), *s = malloc(sizeof(uint16_t) * st * (h + 8));
        const int base = (int)rng_below(&r, 1u << bd), kind = n & 1;
        for (int k = 0; k < st * (h + 8); k++) {
            d[k] = (uint16_t)rand_px(&r, bd, base, kind);
            s[k] = (uint16_t)clampi(d[k] + (int)rng_below(&r, 9) - 4, 0, (1 << bd) - 1);
        }
        int64_t M[49], H[49 * 49];
        if (bd == 8) {
            uint8_t *d8 = malloc(st * (h + 8)), *s8 = malloc(st * (h + 8));
            for (int k = 0; k < st * (h + 8); k++) d8[k] = (uint8_t)d[k], s8[k] = (uint8_t)s[k];
            svt_av1_compute_stats_c(win, d8 + 4 * st + 4, s8 + 4 * st + 4, 0, w, 0, h, st, st, M, H);
            free(d8), free(s8);
        } else
            svt_av1_compute_stats_highbd_c(win, CONVERT_TO_BYTEPTR(d + 4 * st + 4), CONVERT_TO_BYTEPTR(s + 4 * st + 4), 0, w,
                                           0, h, st, st, M, H, (EbBitDepth)bd);
        int32_t *m = meta + 6 * n;
        m[0] = bd, m[1] = win, m[2] = w, m[3] = h, m[4] = st, m[5] = 0;
        char nm[32];
        snprintf(nm, sizeof nm, "dgd%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)(h + 8), (uint32_t)st, d);
        snprintf(nm, sizeof nm, "src%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)(h + 8), (uint32_t)st, s);
        snprintf(nm, sizeof nm, "M%d", n);
        golden_put1(&g, nm, 'q', (uint32_t)(win * win), M);
        snprintf(nm, sizeof nm, "H%d", n);
        golden_put1(&g, nm, 'q', (uint32_t)(win * win * win * win), H);
        free(d), free(s);
    }
    golden_put2(&g, "meta", 'i', N, 6, meta);
    golden_close(&g);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    bind_c_kernels();
    gen_wiener(argv[1]);
    gen_sgr(argv[1]);
    gen_frames(argv[1]);
    gen_stats(argv[1]);
    gen_search(argv[1]);
    printf("lr golden vectors written to %s\n", argv[1]);
    return 0;
}
