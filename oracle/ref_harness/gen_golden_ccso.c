/*
 * gen_golden_ccso.c — CCSO golden vectors (test infrastructure; never shipped).  SURVEY §8(f)4.
 *
 * Links the REFERENCE's own EbCcso.c / EbPickccso.c (compiled from /root/reference by oracle/ref.mk) and records, on
 * deterministic SplitMix64 content:
 *   blk*      the per-block RTCD kernels' C versions (common_dsp_rtcd.h:1025-1090): ccso_derive_src_block_c,
 *             ccso_filter_block_hbd_with_buf_c, ccso_filter_block_hbd_wo_buf_c, compute_distortion_block_c
 *   ext*      extend_ccso_border (EbCcso.c:185-201) of a copied luma plane
 *   srch*     ccso_search (EbPickccso.c:785-815) on a PictureControlSet built here: the three planes' ccso_info and
 *             the block flags it writes into the mode-info grid, then (8-bit) ccso_frame (EbCcso.c:626-678) applying
 *             them to the recon picture
 *   app*      ccso_frame with random ccso_info / block flags (band-offset-only, every filter support, band counts)
 * usage: gen_golden_ccso <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "EbDefinitions.h"
#include "EbPictureControlSet.h"
#include "EbSequenceControlSet.h"
#include "EbCodingUnit.h"
#include "EbCcso.h"
#include "EbPickccso.h"
#include "common_dsp_rtcd.h"
#include "golden_io.h"

#define PAD 5

static void bind_c_kernels(void) {
    ccso_filter_block_hbd_wo_buf   = ccso_filter_block_hbd_wo_buf_c;
    ccso_filter_block_hbd_with_buf = ccso_filter_block_hbd_with_buf_c;
    ccso_derive_src_block          = ccso_derive_src_block_c;
    compute_distortion_block       = compute_distortion_block_c;
    svt_memcpy                     = svt_memcpy_c;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* ---- per-block kernels ---- */
static void block_cases(GoldenFile *g, Rng *r) {
    enum { N = 12 };
    int32_t meta[N][16];
    memset(meta, 0, sizeof meta);
    char nm[40];
    for (int n = 0; n < N; n++) {
        const int bd = n & 1 ? 10 : 8, maxv = (1 << bd) - 1, chroma = (n >> 1) & 1;
        const int hs = chroma, vs = chroma, blk = chroma ? 128 : 256;
        /* a picture a few blocks wide, the block at (x, y) of it (the last block row / column ragged) */
        const int pw = 40 + (int)rng_below(r, 260 - 120 * chroma), ph = 16 + (int)rng_below(r, 48);
        const int x = (int)rng_below(r, 2) * (pw > blk ? blk : 0), y = 0;
        const int lw = pw << hs, lh = ph << vs, es = lw + 2 * PAD, cs = lw;
        uint16_t *ext = malloc(sizeof(uint16_t) * (size_t)es * (lh + 2 * PAD));
        /* smooth content with edges so every class occurs */
        for (int i = 0; i < es * (lh + 2 * PAD); i++)
            ext[i] = (uint16_t)clampi((int)((i % es) * 3 + (i / es) * 2) % (maxv + 1) + (int)rng_below(r, 40) - 20, 0,
                                      maxv);
        const uint16_t *src = ext + PAD * es + PAD;
        const int       sup = (int)rng_below(r, 6), qs = (int[]){16, 8, 32, 64}[rng_below(r, 4)];
        const int       clf = (int)rng_below(r, 2), bo = n % 5 == 4, band_log2 = (int)rng_below(r, bo ? 8 : 4);
        int             loc[2];
        derive_ccso_sample_pos(loc, es, (uint8_t)sup);
        uint8_t *c0 = calloc((size_t)cs * lh, 1), *c1 = calloc((size_t)cs * lh, 1);
        ccso_derive_src_block_c(src, c0, c1, es, cs, x, y, pw, ph, hs, vs, qs, -qs, loc, blk, clf);
        int8_t lut[2048];
        for (int i = 0; i < 2048; i++) lut[i] = (int8_t)((int)rng_below(r, 18) - 10);
        uint16_t *dst = malloc(sizeof(uint16_t) * (size_t)cs * ph), *dst0 = malloc(sizeof(uint16_t) * (size_t)cs * ph);
        for (int i = 0; i < cs * ph; i++) dst[i] = dst0[i] = (uint16_t)rng_below(r, maxv + 1);
        uint16_t *dst2 = malloc(sizeof(uint16_t) * (size_t)cs * ph);
        memcpy(dst2, dst0, sizeof(uint16_t) * (size_t)cs * ph);
        ccso_filter_block_hbd_with_buf_c(src, dst, c0, c1, es, cs, cs, x, y, pw, ph, lut, blk, hs, vs, maxv,
                                         (uint8_t)(bd - band_log2), (uint8_t)bo);
        int cls[2] = {0, 0};
        ccso_filter_block_hbd_wo_buf_c(src, dst2, x, y, pw, ph, cls, lut, es, cs, hs, vs, qs, -qs, loc, maxv, blk,
                                       band_log2 == 0, (uint8_t)(bd - band_log2), clf, (uint8_t)bo);
        const int      log2 = chroma ? 7 : 8;
        const uint64_t ssd  = compute_distortion_block_c(dst0, cs, dst, cs, x, y, log2, ph, pw);
        snprintf(nm, sizeof nm, "blk_ext%d", n), golden_put1(g, nm, 'H', (uint32_t)(es * (lh + 2 * PAD)), ext);
        snprintf(nm, sizeof nm, "blk_cls0_%d", n), golden_put1(g, nm, 'B', (uint32_t)(cs * lh), c0);
        snprintf(nm, sizeof nm, "blk_cls1_%d", n), golden_put1(g, nm, 'B', (uint32_t)(cs * lh), c1);
        snprintf(nm, sizeof nm, "blk_lut%d", n), golden_put1(g, nm, 'b', 2048, lut);
        snprintf(nm, sizeof nm, "blk_dst0_%d", n), golden_put1(g, nm, 'H', (uint32_t)(cs * ph), dst0);
        snprintf(nm, sizeof nm, "blk_with%d", n), golden_put1(g, nm, 'H', (uint32_t)(cs * ph), dst);
        snprintf(nm, sizeof nm, "blk_wo%d", n), golden_put1(g, nm, 'H', (uint32_t)(cs * ph), dst2);
        snprintf(nm, sizeof nm, "blk_ssd%d", n), golden_put1(g, nm, 'Q', 1, &ssd);
        int32_t *m = meta[n];
        m[0] = pw, m[1] = ph, m[2] = x, m[3] = y, m[4] = hs, m[5] = vs, m[6] = blk, m[7] = bd, m[8] = sup, m[9] = qs;
        m[10] = clf, m[11] = bo, m[12] = band_log2, m[13] = es, m[14] = cs, m[15] = loc[0];
        free(ext), free(c0), free(c1), free(dst), free(dst0), free(dst2);
    }
    uint32_t dims[2] = {N, 16};
    golden_put(g, "blk_meta", 'i', 2, dims, meta);
}

/* ---- frame-level: a PictureControlSet of the fields ccso_search / ccso_frame read ---- */
typedef struct {
    SequenceControlSet      *scs;
    PictureParentControlSet *ppcs;
    PictureControlSet       *pcs;
    Av1Common               *cm;
    EncDecSet               *eds;
    MbModeInfo              *cells;
    EbPictureBufferDesc     *recon;
    int                      mi_rows, mi_cols;
} Pic;

static EbErrorType new_pic_desc(EbPictureBufferDesc **out, int w, int h, int hbd) {
    EbPictureBufferDescInitData d;
    memset(&d, 0, sizeof d);
    d.max_width          = (uint16_t)w;
    d.max_height         = (uint16_t)h;
    d.bit_depth          = hbd ? EB_TEN_BIT : EB_EIGHT_BIT;
    d.color_format       = EB_YUV420;
    d.buffer_enable_mask = PICTURE_BUFFER_DESC_FULL_MASK;
    d.left_padding = d.right_padding = d.top_padding = d.bot_padding = 32;
    EbPictureBufferDesc *p;
    EB_NEW(p, svt_recon_picture_buffer_desc_ctor, (EbPtr)&d);
    *out = p;
    return EB_ErrorNone;
}
static EbPictureBufferDesc *new_pic(int w, int h, int hbd) {
    EbPictureBufferDesc *p = NULL;
    if (new_pic_desc(&p, w, h, hbd) != EB_ErrorNone) exit(3);
    return p;
}

static uint8_t *plane8(EbPictureBufferDesc *p, int pl, int *stride) {
    const int st = pl == 0 ? p->stride_y : pl == 1 ? p->stride_cb : p->stride_cr;
    uint8_t  *b  = pl == 0 ? p->buffer_y : pl == 1 ? p->buffer_cb : p->buffer_cr;
    const int ox = pl ? p->org_x / 2 : p->org_x, oy = pl ? p->org_y / 2 : p->org_y;
    *stride      = st;
    return b + (size_t)oy * st + ox;
}

static void pic_init(Pic *P, int W, int H, int bd, int q) {
    memset(P, 0, sizeof *P);
    P->scs = calloc(1, sizeof *P->scs), P->ppcs = calloc(1, sizeof *P->ppcs), P->pcs = calloc(1, sizeof *P->pcs);
    P->cm = calloc(1, sizeof *P->cm), P->eds = calloc(1, sizeof *P->eds);
    P->pcs->scs = P->ppcs->scs = P->scs;
    P->pcs->ppcs = P->ppcs, P->ppcs->av1_cm = P->cm, P->ppcs->enc_dec_ptr = P->eds, P->cm->child_pcs = P->pcs;
    P->scs->seq_header.sb_size                 = BLOCK_64X64;
    P->scs->is_16bit_pipeline                  = (uint8_t)(bd > 8);
    P->scs->static_config.encoder_bit_depth    = (uint32_t)bd;
    P->scs->static_config.encoder_color_format = EB_YUV420;
    P->scs->max_input_luma_width               = (uint16_t)W;
    P->scs->max_input_luma_height              = (uint16_t)H;
    P->scs->seq_header.color_config.mono_chrome = 0;
    P->ppcs->render_width = (uint16_t)W, P->ppcs->render_height = (uint16_t)H;
    P->ppcs->frm_hdr.quantization_params.base_q_idx = (uint8_t)q;
    P->mi_cols = ((W + 7) & ~7) >> 2, P->mi_rows = ((H + 7) & ~7) >> 2;
    P->cm->mi_rows = P->mi_rows, P->cm->mi_cols = P->mi_cols, P->cm->mi_stride = P->mi_cols;
    P->cells                = calloc((size_t)P->mi_rows * P->mi_cols, sizeof(MbModeInfo));
    ModeInfo **grid         = calloc((size_t)P->mi_rows * P->mi_cols, sizeof(ModeInfo *));
    for (int k = 0; k < P->mi_rows * P->mi_cols; k++) grid[k] = (ModeInfo *)&P->cells[k];
    P->pcs->mi_grid_base = grid;
    P->pcs->mi_stride    = (uint16_t)P->mi_cols;
    P->recon             = new_pic(W, H, bd > 8);
    if (bd > 8) P->eds->recon_pic_16bit = P->recon;
    else P->eds->recon_pic = P->recon;
}

static void pd_init(MacroblockdPlane pd[3]) {
    memset(pd, 0, sizeof(MacroblockdPlane) * 3);
    for (int p = 0; p < 3; p++) pd[p].subsampling_x = pd[p].subsampling_y = p > 0, pd[p].is_16bit = 0;
}

/* the block flags of one plane as the search writes them into the mode-info grid (EbPickccso.c:731-751) */
static void flags_get(Pic *P, int plane, int nvfb, int nhfb, uint8_t *f) {
    for (int y = 0; y < nvfb; y++)
        for (int x = 0; x < nhfb; x++) {
            const MbModeInfo *m = &P->cells[64 * y * P->mi_cols + 64 * x];
            f[y * nhfb + x]     = plane == 0 ? m->ccso_blk_y : plane == 1 ? m->ccso_blk_u : m->ccso_blk_v;
        }
}
static void flags_set(Pic *P, int plane, int nvfb, int nhfb, const uint8_t *f) {
    for (int y = 0; y < nvfb; y++)
        for (int x = 0; x < nhfb; x++) {
            MbModeInfo *m = &P->cells[64 * y * P->mi_cols + 64 * x];
            if (plane == 0) m->ccso_blk_y = f[y * nhfb + x];
            else if (plane == 1) m->ccso_blk_u = f[y * nhfb + x];
            else m->ccso_blk_v = f[y * nhfb + x];
        }
}
static void grid_dims(const Pic *P, int plane, int *nvfb, int *nhfb) {
    const int ss = plane > 0, unit = (plane ? 128 : 256) >> 2;
    *nvfb = ((P->mi_rows >> ss) + unit - 1) / unit, *nhfb = ((P->mi_cols >> ss) + unit - 1) / unit;
}

/* org / rec planes (stride W, H rows each, chroma in the top-left (W >> 1) x (H >> 1)): value-noise content with a
 * coding-error model that CCSO can partly undo (a band- and edge-dependent bias), dark and bright areas for the clamps */
static void content(Rng *r, int W, int H, int bd, uint16_t *org[3], uint16_t *rec[3], uint16_t *pre_y, int bias) {
    const int maxv = (1 << bd) - 1, sh = bd - 8;
    for (int p = 0; p < 3; p++) {
        const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H, g = 16;
        const int gw = pw / g + 2, gh = ph / g + 2;
        int      *kn = malloc(sizeof(int) * gw * gh);
        for (int i = 0; i < gw * gh; i++) kn[i] = (int)rng_below(r, 256);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) {
                const int gx = x / g, gy = y / g, fx = x % g, fy = y % g;
                int v = (kn[gy * gw + gx] * (g - fx) * (g - fy) + kn[gy * gw + gx + 1] * fx * (g - fy) +
                         kn[(gy + 1) * gw + gx] * (g - fx) * fy + kn[(gy + 1) * gw + gx + 1] * fx * fy) / (g * g);
                if (x < pw / 8) v = v / 16;                         /* dark strip: the low clamp */
                if (x >= pw - pw / 8) v = 255 - (255 - v) / 16;     /* bright strip: the high clamp */
                v = clampi((v << sh) + (int)rng_below(r, 5 << sh) - (2 << sh), 0, maxv);
                org[p][(size_t)y * W + x] = (uint16_t)v;
            }
        free(kn);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) {
                const int o  = org[p][(size_t)y * W + x];
                const int gx = x + 1 < pw ? org[p][(size_t)y * W + x + 1] - o : 0;
                int       e  = (int)rng_below(r, 7) - 3;
                if (o > (maxv * 3) / 4) e -= bias;            /* band-dependent error */
                if (gx > (8 << sh)) e += bias;                /* edge-dependent error */
                if (gx < -(8 << sh)) e -= bias;
                rec[p][(size_t)y * W + x] = (uint16_t)clampi(o + (e << sh), 0, maxv);
            }
    }
    for (int i = 0; i < W * H; i++) pre_y[i] = (uint16_t)clampi(rec[0][i] + (int)rng_below(r, 3) - 1, 0, maxv);
}

/* one plane's pw x ph samples (stride W), 8-bit planes as bytes */
static void put_plane(GoldenFile *g, const char *nm, const uint16_t *a, int W, int pw, int ph, int bd) {
    void *b = malloc((size_t)pw * ph * 2);
    for (int y = 0; y < ph; y++)
        for (int x = 0; x < pw; x++) {
            if (bd == 8) ((uint8_t *)b)[(size_t)y * pw + x] = (uint8_t)a[(size_t)y * W + x];
            else ((uint16_t *)b)[(size_t)y * pw + x] = a[(size_t)y * W + x];
        }
    golden_put2(g, nm, bd == 8 ? 'B' : 'H', (uint32_t)ph, (uint32_t)pw, b);
    free(b);
}

static void put_params(GoldenFile *g, const char *tag, int n, const FrameHeader *fh, int plane) {
    char    nm[48];
    int32_t f[7] = {fh->ccso_info.ccso_enable[plane], fh->ccso_info.ccso_bo_only[plane], fh->ccso_info.quant_idx[plane],
                    fh->ccso_info.ext_filter_support[plane], fh->ccso_info.max_band_log2[plane],
                    fh->ccso_info.edge_clf[plane], 0};
    snprintf(nm, sizeof nm, "%s_prm%d_%d", tag, n, plane), golden_put1(g, nm, 'i', 7, f);
    snprintf(nm, sizeof nm, "%s_lut%d_%d", tag, n, plane), golden_put1(g, nm, 'b', 2048, fh->ccso_info.filter_offset[plane]);
}

static void emit_recon8(GoldenFile *g, const char *tag, int n, Pic *P, int W, int H) {
    char nm[48];
    for (int p = 0; p < 3; p++) {
        const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H;
        int       st;
        uint8_t  *b = plane8(P->recon, p, &st), *a = malloc((size_t)pw * ph);
        for (int y = 0; y < ph; y++) memcpy(a + (size_t)y * pw, b + (size_t)y * st, pw);
        snprintf(nm, sizeof nm, "%s_out%d_%d", tag, n, p), golden_put2(g, nm, 'B', (uint32_t)ph, (uint32_t)pw, a);
        free(a);
    }
}

static void load_recon8(Pic *P, uint16_t *rec[3], int W, int H) {
    for (int p = 0; p < 3; p++) {
        const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H;
        int       st;
        uint8_t  *b = plane8(P->recon, p, &st);
        for (int y = 0; y < ph; y++)
            for (int x = 0; x < pw; x++) b[(size_t)y * st + x] = (uint8_t)rec[p][(size_t)y * W + x];
    }
}

static uint16_t *make_ext(const uint16_t *pre_y, int W, int H) {
    MacroblockdPlane pd[3];
    pd_init(pd);
    pd[0].dst.width = W, pd[0].dst.height = H;
    const int es  = W + 2 * PAD;
    uint16_t *ext = calloc((size_t)es * (H + 2 * PAD), sizeof(uint16_t));
    for (int y = 0; y < H; y++) memcpy(ext + (size_t)(y + PAD) * es + PAD, pre_y + (size_t)y * W, 2 * (size_t)W);
    extend_ccso_border(ext, PAD, pd);
    return ext;
}

static void search_cases(GoldenFile *g, Rng *r) {
    /* {W, H, bd, q, rdmult, bias} */
    static const int cs[][6] = {{320, 192, 8, 100, 2600, 3},   {300, 264, 8, 60, 900, 2},      {257, 136, 8, 30, 4000, 3},
                                {264, 264, 10, 120, 5000, 2},  {200, 120, 8, 150, 300, 4},     {192, 128, 8, 63, 3000000, 0},
                                {64, 64, 8, 63, 40000000, 2},  {264, 200, 10, 90, 700, 3},     {136, 72, 8, 255, 20000, 1}};
    const int n_cases = (int)(sizeof cs / sizeof cs[0]);
    int32_t   meta[16][6];
    char      nm[48];
    for (int n = 0; n < n_cases; n++) {
        const int W = cs[n][0], H = cs[n][1], bd = cs[n][2], q = cs[n][3], rdmult = cs[n][4], bias = cs[n][5];
        memcpy(meta[n], cs[n], sizeof meta[n]);
        uint16_t *org[3], *rec[3], *pre = malloc(2 * (size_t)W * H);
        for (int p = 0; p < 3; p++) org[p] = calloc((size_t)W * H, 2), rec[p] = calloc((size_t)W * H, 2);
        content(r, W, H, bd, org, rec, pre, bias);
        uint16_t *ext = make_ext(pre, W, H);
        Pic       P;
        pic_init(&P, W, H, bd, q);
        MacroblockdPlane pd[3];
        pd_init(pd);
        for (int p = 0; p < 3; p++) {
            const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H;
            snprintf(nm, sizeof nm, "srch_org%d_%d", n, p), put_plane(g, nm, org[p], W, pw, ph, bd);
            snprintf(nm, sizeof nm, "srch_rec%d_%d", n, p), put_plane(g, nm, rec[p], W, pw, ph, bd);
        }
        snprintf(nm, sizeof nm, "srch_pre%d", n), put_plane(g, nm, pre, W, W, H, bd);
        if (n == 0 || bd > 8) /* extend_ccso_border's output, once per bit depth */
            snprintf(nm, sizeof nm, "srch_ext%d", n),
                golden_put2(g, nm, 'H', (uint32_t)(H + 2 * PAD), (uint32_t)(W + 2 * PAD), ext);
        ccso_search(P.pcs, pd, rdmult, ext, rec, org);
        const FrameHeader *fh = &P.ppcs->frm_hdr;
        for (int p = 0; p < 3; p++) {
            int nvfb, nhfb;
            grid_dims(&P, p, &nvfb, &nhfb);
            uint8_t *f = calloc((size_t)nvfb * nhfb, 1);
            if (fh->ccso_info.ccso_enable[p]) flags_get(&P, p, nvfb, nhfb, f);
            put_params(g, "srch", n, fh, p);
            snprintf(nm, sizeof nm, "srch_flags%d_%d", n, p), golden_put2(g, nm, 'B', (uint32_t)nvfb, (uint32_t)nhfb, f);
            free(f);
        }
        int32_t ff = fh->ccso_info.ccso_frame_flag;
        snprintf(nm, sizeof nm, "srch_frame_flag%d", n), golden_put1(g, nm, 'i', 1, &ff);
        if (bd == 8) { /* ccso_frame applies the search's result to the recon picture (8-bit buffers, EbCcso.c:638-677) */
            load_recon8(&P, rec, W, H);
            pd_init(pd);
            ccso_frame(P.recon, P.pcs, pd, ext);
            emit_recon8(g, "srch", n, &P, W, H);
        }
        for (int p = 0; p < 3; p++) free(org[p]), free(rec[p]);
        free(pre), free(ext);
        printf("search case %d: %dx%d %d-bit -> enable %d %d %d\n", n, W, H, bd, fh->ccso_info.ccso_enable[0],
               fh->ccso_info.ccso_enable[1], fh->ccso_info.ccso_enable[2]);
    }
    uint32_t dims[2] = {(uint32_t)n_cases, 6};
    golden_put(g, "srch_meta", 'i', 2, dims, meta);
}

static void apply_cases(GoldenFile *g, Rng *r) {
    static const int cs[][2] = {{320, 144}, {520, 96}, {257, 130}, {136, 296}, {96, 64}};
    const int        n_cases = (int)(sizeof cs / sizeof cs[0]);
    int32_t          meta[8][2];
    char             nm[48];
    for (int n = 0; n < n_cases; n++) {
        const int W = cs[n][0], H = cs[n][1];
        meta[n][0] = W, meta[n][1] = H;
        uint16_t *org[3], *rec[3], *pre = malloc(2 * (size_t)W * H);
        for (int p = 0; p < 3; p++) org[p] = calloc((size_t)W * H, 2), rec[p] = calloc((size_t)W * H, 2);
        content(r, W, H, 8, org, rec, pre, 2);
        uint16_t *ext = make_ext(pre, W, H);
        Pic       P;
        pic_init(&P, W, H, 8, 100);
        FrameHeader *fh = &P.ppcs->frm_hdr;
        for (int p = 0; p < 3; p++) {
            const int k = n * 3 + p;
            fh->ccso_info.ccso_enable[p]        = k % 7 != 5;
            fh->ccso_info.ccso_bo_only[p]       = (uint8_t)(k % 4 == 3);
            fh->ccso_info.quant_idx[p]          = (uint8_t)rng_below(r, 4);
            fh->ccso_info.ext_filter_support[p] = (uint8_t)(k % 6);
            fh->ccso_info.max_band_log2[p]      = (int)rng_below(r, fh->ccso_info.ccso_bo_only[p] ? 8 : 4);
            fh->ccso_info.edge_clf[p]           = (uint8_t)rng_below(r, 2);
            for (int i = 0; i < 2048; i++) fh->ccso_info.filter_offset[p][i] = (int8_t)((int)rng_below(r, 18) - 10);
            int nvfb, nhfb;
            grid_dims(&P, p, &nvfb, &nhfb);
            uint8_t *f = malloc((size_t)nvfb * nhfb);
            for (int i = 0; i < nvfb * nhfb; i++) f[i] = (uint8_t)(rng_below(r, 4) != 0);
            flags_set(&P, p, nvfb, nhfb, f);
            put_params(g, "app", n, fh, p);
            snprintf(nm, sizeof nm, "app_flags%d_%d", n, p), golden_put2(g, nm, 'B', (uint32_t)nvfb, (uint32_t)nhfb, f);
            free(f);
        }
        load_recon8(&P, rec, W, H);
        for (int p = 0; p < 3; p++) {
            const int pw = p ? W >> 1 : W, ph = p ? H >> 1 : H;
            snprintf(nm, sizeof nm, "app_in%d_%d", n, p), put_plane(g, nm, rec[p], W, pw, ph, 8);
        }
        snprintf(nm, sizeof nm, "app_pre%d", n), put_plane(g, nm, pre, W, W, H, 8);
        MacroblockdPlane pd[3];
        pd_init(pd);
        ccso_frame(P.recon, P.pcs, pd, ext);
        emit_recon8(g, "app", n, &P, W, H);
        for (int p = 0; p < 3; p++) free(org[p]), free(rec[p]);
        free(pre), free(ext);
    }
    uint32_t dims[2] = {(uint32_t)n_cases, 2};
    golden_put(g, "app_meta", 'i', 2, dims, meta);
}

/* the reference's CPU cost of one frame's ccso_search (+ ccso_frame at 8 bits) on the golden content model: the
 * cpu_baseline of scripts/r6/ccso_perf.py (kind "reference", one thread) */
void     ccso_filter_block_hbd_wo_buf_avx2(const uint16_t *src_y, uint16_t *dst_yuv, const int x, const int y,
                                           const int pic_width, const int pic_height, int *src_cls,
                                           const int8_t *offset_buf, const int src_y_stride, const int dst_stride,
                                           const int y_uv_hscale, const int y_uv_vscale, const int thr,
                                           const int neg_thr, const int *src_loc, const int max_val, const int blk_size,
                                           const bool isSingleBand, const uint8_t shift_bits, const int edge_clf,
                                           const uint8_t ccso_bo_only);
void     ccso_derive_src_block_avx2(const uint16_t *src_y, uint8_t *const src_cls0, uint8_t *const src_cls1,
                                    const int src_y_stride, const int ccso_stride, const int x, const int y,
                                    const int pic_width, const int pic_height, const int y_uv_hscale,
                                    const int y_uv_vscale, const int qstep, const int neg_qstep, const int *src_loc,
                                    const int blk_size, const int edge_clf);
void     ccso_filter_block_hbd_with_buf_avx2(const uint16_t *src_y, uint16_t *dst_yuv, const uint8_t *src_cls0,
                                             const uint8_t *src_cls1, const int src_y_stride, const int dst_stride,
                                             const int ccso_stride, const int x, const int y, const int pic_width,
                                             const int pic_height, const int8_t *filter_offset, const int blk_size,
                                             const int y_uv_hscale, const int y_uv_vscale, const int max_val,
                                             const uint8_t shift_bits, const uint8_t ccso_bo_only);
uint64_t compute_distortion_block_avx2(const uint16_t *org, const int org_stride, const uint16_t *rec16,
                                       const int rec_stride, const int x, const int y, const int log2_filter_unit_size,
                                       const int height, const int width);

static int bench(int W, int H, int bd, int reps, int avx2) {
    bind_c_kernels();
    if (avx2) { /* the bindings setup_common_rtcd_internal makes on an AVX2 host (common_dsp_rtcd.c:637-639) */
        ccso_filter_block_hbd_wo_buf   = ccso_filter_block_hbd_wo_buf_avx2;
        ccso_filter_block_hbd_with_buf = ccso_filter_block_hbd_with_buf_avx2;
        ccso_derive_src_block          = ccso_derive_src_block_avx2;
        compute_distortion_block       = compute_distortion_block_avx2;
    }
    Rng       r = {0x4343534F0000BE01ull};
    uint16_t *org[3], *rec[3], *pre = malloc(2 * (size_t)W * H);
    for (int p = 0; p < 3; p++) org[p] = calloc((size_t)W * H, 2), rec[p] = calloc((size_t)W * H, 2);
    content(&r, W, H, bd, org, rec, pre, 2);
    uint16_t *ext = make_ext(pre, W, H);
    double    best = 1e30, best_apply = 1e30;
    for (int k = 0; k < reps; k++) {
        Pic P;
        pic_init(&P, W, H, bd, 100);
        MacroblockdPlane pd[3];
        pd_init(pd);
        struct timespec t0, t1, t2;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        ccso_search(P.pcs, pd, 1500, ext, rec, org);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        const double ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
        best            = ms < best ? ms : best;
        if (bd == 8) {
            load_recon8(&P, rec, W, H);
            pd_init(pd);
            ccso_frame(P.recon, P.pcs, pd, ext);
            clock_gettime(CLOCK_MONOTONIC, &t2);
            const double ma = (t2.tv_sec - t1.tv_sec) * 1e3 + (t2.tv_nsec - t1.tv_nsec) * 1e-6;
            best_apply      = ma < best_apply ? ma : best_apply;
        }
        printf("rep %d: search %.1f ms enable %d %d %d\n", k, ms, P.ppcs->frm_hdr.ccso_info.ccso_enable[0],
               P.ppcs->frm_hdr.ccso_info.ccso_enable[1], P.ppcs->frm_hdr.ccso_info.ccso_enable[2]);
    }
    printf("{\"w\": %d, \"h\": %d, \"bd\": %d, \"search_ms\": %.3f, \"apply_ms\": %.3f, \"threads\": 1, "
           "\"kernels\": \"%s\"}\n", W, H, bd, best, bd == 8 ? best_apply : -1.0, avx2 ? "avx2" : "c");
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "bench"))
        return bench(argc > 2 ? atoi(argv[2]) : 1920, argc > 3 ? atoi(argv[3]) : 1080, argc > 4 ? atoi(argv[4]) : 8,
                     argc > 5 ? atoi(argv[5]) : 1, argc > 6 && !strcmp(argv[6], "avx2"));
    const char *dir = argc > 1 ? argv[1] : "tests/golden";
    char        path[512];
    snprintf(path, sizeof path, "%s/ccso.bin", dir);
    bind_c_kernels();
    GoldenFile g = golden_open(path);
    Rng        r = {0x4343534F00000001ull};
    block_cases(&g, &r);
    apply_cases(&g, &r);
    search_cases(&g, &r);
    golden_close(&g);
    printf("wrote %s\n", path);
    return 0;
}
