/*
 * gen_golden_dlf.c — deblocking golden-vector generator (test infrastructure; never shipped).
 *
 * Links the REFERENCE's own deblocking C (EbDeblockingCommon.c, EbDeblockingFilter.c, compiled from
 * /root/reference by oracle/ref.mk) and records its outputs on deterministic SplitMix64 inputs:
 *   dlf_lpf.bin    every svt_aom_lpf_* / svt_aom_highbd_lpf_* C kernel (bd 8/10/12) on windows that
 *                  mix noise, flat areas and steps (sweep after the reference's test/LoopFilterTest.cc)
 *   dlf_frame.bin  svt_av1_loop_filter_frame on whole frames with random partitions / transform
 *                  depths / skip / refs / modes / segments, sharpness, mode-ref deltas and
 *                  segmentation features, 8-bit and 16-bit pipelines
 * usage: gen_golden_dlf <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbPictureControlSet.h"
#include "EbSequenceControlSet.h"
#include "EbDeblockingFilter.h"
#include "common_dsp_rtcd.h"
#include "golden_io.h"

void svt_av1_loop_filter_init(PictureControlSet *pcs);
void svt_av1_loop_filter_frame(EbPictureBufferDesc *frame_buffer, PictureControlSet *pcs, int32_t plane_start,
                               int32_t plane_end);

static void bind_c_kernels(void) {
    svt_aom_lpf_horizontal_4         = svt_aom_lpf_horizontal_4_c;
    svt_aom_lpf_horizontal_6         = svt_aom_lpf_horizontal_6_c;
    svt_aom_lpf_horizontal_8         = svt_aom_lpf_horizontal_8_c;
    svt_aom_lpf_horizontal_14        = svt_aom_lpf_horizontal_14_c;
    svt_aom_lpf_vertical_4           = svt_aom_lpf_vertical_4_c;
    svt_aom_lpf_vertical_6           = svt_aom_lpf_vertical_6_c;
    svt_aom_lpf_vertical_8           = svt_aom_lpf_vertical_8_c;
    svt_aom_lpf_vertical_14          = svt_aom_lpf_vertical_14_c;
    svt_aom_highbd_lpf_horizontal_4  = svt_aom_highbd_lpf_horizontal_4_c;
    svt_aom_highbd_lpf_horizontal_6  = svt_aom_highbd_lpf_horizontal_6_c;
    svt_aom_highbd_lpf_horizontal_8  = svt_aom_highbd_lpf_horizontal_8_c;
    svt_aom_highbd_lpf_horizontal_14 = svt_aom_highbd_lpf_horizontal_14_c;
    svt_aom_highbd_lpf_vertical_4    = svt_aom_highbd_lpf_vertical_4_c;
    svt_aom_highbd_lpf_vertical_6    = svt_aom_highbd_lpf_vertical_6_c;
    svt_aom_highbd_lpf_vertical_8    = svt_aom_highbd_lpf_vertical_8_c;
    svt_aom_highbd_lpf_vertical_14   = svt_aom_highbd_lpf_vertical_14_c;
    svt_log2f                        = svt_aom_log2f_32; /* C; used for the SB grid */
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* ------------------------------------------------------------------------------------------- */
/* kernel level: 16x16 window, edge through the centre (row/col 8), pitch 16                      */
/* ------------------------------------------------------------------------------------------- */
#define LPF_N 250
#define WIN 16

static void fill_window(Rng *r, uint16_t *w, int bd, int kind) {
    const int one = 1 << (bd - 8), maxv = (1 << bd) - 1;
    const int base = (int)rng_below(r, (uint32_t)maxv + 1);
    /* kind 0: random; 1: flat + step across the centre; 2: flat + noise 0/1 unit; 3: ramp */
    const int step = ((int)rng_below(r, 13) - 6) * one;
    for (int y = 0; y < WIN; y++)
        for (int x = 0; x < WIN; x++) {
            int v;
            if (kind == 0)
                v = (int)rng_below(r, (uint32_t)maxv + 1);
            else if (kind == 1)
                v = base + ((x >= 8) != (y >= 8) ? step : 0) + (int)rng_below(r, 2) * one;
            else if (kind == 2)
                v = base + ((int)rng_below(r, 3) - 1) * one;
            else
                v = base + (x + y) * (int)rng_below(r, 3) * one / 2 + (x >= 8 ? step : 0);
            w[y * WIN + x] = (uint16_t)clampi(v, 0, maxv);
        }
}

typedef void (*Lpf8Fn)(uint8_t *, int32_t, const uint8_t *, const uint8_t *, const uint8_t *);
typedef void (*Lpf16Fn)(uint16_t *, int32_t, const uint8_t *, const uint8_t *, const uint8_t *, int32_t);

static void gen_lpf(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/dlf_lpf.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0xD1F0000000000001ull};
    /* function index f: 0..3 horizontal 4/6/8/14, 4..7 vertical 4/6/8/14 */
    Lpf8Fn  f8[8]  = {svt_aom_lpf_horizontal_4_c, svt_aom_lpf_horizontal_6_c, svt_aom_lpf_horizontal_8_c,
                      svt_aom_lpf_horizontal_14_c, svt_aom_lpf_vertical_4_c, svt_aom_lpf_vertical_6_c,
                      svt_aom_lpf_vertical_8_c, svt_aom_lpf_vertical_14_c};
    Lpf16Fn f16[8] = {svt_aom_highbd_lpf_horizontal_4_c, svt_aom_highbd_lpf_horizontal_6_c,
                      svt_aom_highbd_lpf_horizontal_8_c, svt_aom_highbd_lpf_horizontal_14_c,
                      svt_aom_highbd_lpf_vertical_4_c,   svt_aom_highbd_lpf_vertical_6_c,
                      svt_aom_highbd_lpf_vertical_8_c,   svt_aom_highbd_lpf_vertical_14_c};
    /* records: meta[i] = {bd (8 = 8-bit kernels, 108 = highbd at bd 8, 10, 12), fn, blimit, limit, thresh} */
    const int bds[4] = {8, 108, 10, 12};
    const int total  = 4 * 8 * LPF_N;
    int32_t  *meta   = malloc(sizeof(int32_t) * 5 * total);
    /* stored as the 4 sample lines crossing the edge, 16 samples each (edge between 7 and 8) */
    uint16_t *in     = malloc(sizeof(uint16_t) * 4 * WIN * total);
    uint16_t *out    = malloc(sizeof(uint16_t) * 4 * WIN * total);
    int       n      = 0;
    for (int b = 0; b < 4; b++)
        for (int f = 0; f < 8; f++)
            for (int i = 0; i < LPF_N; i++, n++) {
                const int bd = bds[b] == 108 ? 8 : bds[b];
                /* thresholds as the encoder builds them: lvl -> mblim/lim, hev = lvl >> 4 (some fully random) */
                uint8_t bl, li, th;
                if (i % 4 == 3) {
                    bl = (uint8_t)rng_below(&r, 3 * 63 + 5);
                    li = (uint8_t)rng_below(&r, 64);
                    th = (uint8_t)rng_below(&r, 64);
                } else {
                    const int lvl = (int)rng_below(&r, 64), sh = (int)rng_below(&r, 8);
                    int       bil = lvl >> ((sh > 0) + (sh > 4));
                    if (sh > 0 && bil > 9 - sh) bil = 9 - sh;
                    if (bil < 1) bil = 1;
                    li = (uint8_t)bil;
                    bl = (uint8_t)(2 * (lvl + 2) + bil);
                    th = (uint8_t)(lvl >> 4);
                }
                uint8_t blv[16], liv[16], thv[16];
                memset(blv, bl, 16);
                memset(liv, li, 16);
                memset(thv, th, 16);
                uint16_t w[WIN * WIN], o[WIN * WIN];
                fill_window(&r, w, bd, i % 4 == 3 ? 0 : (int)rng_below(&r, 4));
                memcpy(o, w, sizeof(uint16_t) * WIN * WIN);
                if (bds[b] == 8) {
                    uint8_t w8[WIN * WIN];
                    for (int k = 0; k < WIN * WIN; k++) w8[k] = (uint8_t)o[k];
                    f8[f](w8 + 8 * WIN + 8, WIN, blv, liv, thv);
                    for (int k = 0; k < WIN * WIN; k++) o[k] = w8[k];
                } else
                    f16[f](o + 8 * WIN + 8, WIN, blv, liv, thv, bd);
                for (int l = 0; l < 4; l++)
                    for (int k = 0; k < WIN; k++) {
                        const int idx = f < 4 ? k * WIN + 8 + l : (8 + l) * WIN + k;
                        in[((size_t)n * 4 + l) * WIN + k]  = w[idx];
                        out[((size_t)n * 4 + l) * WIN + k] = o[idx];
                    }
                int32_t *m = meta + 5 * n;
                m[0] = bds[b], m[1] = f, m[2] = bl, m[3] = li, m[4] = th;
            }
    golden_put2(&g, "meta", 'i', (uint32_t)total, 5, meta);
    uint32_t dims[3] = {(uint32_t)total, 4, WIN};
    golden_put(&g, "in", 'H', 3, dims, in);
    golden_put(&g, "out", 'H', 3, dims, out);
    golden_close(&g);
    free(meta);
    free(in);
    free(out);
}

/* ------------------------------------------------------------------------------------------- */
/* frame level                                                                                   */
/* ------------------------------------------------------------------------------------------- */
typedef struct FrameCase {
    int w, h, bd, pipe16, plane_start, plane_end;
    int fl0, fl1, flu, flv, sharp, mrd, seg;
} FrameCase;

static int bsize_of(int w, int h) {
    for (int b = 0; b < BlockSizeS_ALL; b++)
        if (block_size_wide[b] == w && block_size_high[b] == h)
            return b;
    return -1;
}

typedef struct Grid {
    MbModeInfo *blocks;
    int         nblocks, cap;
    ModeInfo  **cells; /* mi_rows * mi_cols pointers into blocks (the reference's mi_grid_base) */
    int         mi_rows, mi_cols;
    Rng        *r;
    int         seg;
} Grid;

static void place(Grid *G, int mi_r, int mi_c, int bw, int bh) {
    if (mi_r >= G->mi_rows || mi_c >= G->mi_cols)
        return;
    MbModeInfo *m = &G->blocks[G->nblocks++];
    memset(m, 0, sizeof(*m));
    Rng *r              = G->r;
    m->block_mi.bsize   = (BlockSize)bsize_of(bw, bh);
    const int inter     = rng_below(r, 10) >= 3;
    m->block_mi.ref_frame[0] = inter ? (MvReferenceFrame)(1 + rng_below(r, 7)) : INTRA_FRAME;
    m->block_mi.mode    = (PredictionMode)(inter ? 13 + rng_below(r, 12) : rng_below(r, 13));
    m->block_mi.skip    = rng_below(r, 2);
    m->block_mi.tx_depth = (uint8_t)rng_below(r, 3);
    m->block_mi.segment_id = G->seg ? (uint8_t)rng_below(r, 8) : 0;
    for (int y = 0; y < bh / 4; y++)
        for (int x = 0; x < bw / 4; x++)
            if (mi_r + y < G->mi_rows && mi_c + x < G->mi_cols)
                G->cells[(mi_r + y) * G->mi_cols + mi_c + x] = (ModeInfo *)m;
}

static void partition(Grid *G, int mi_r, int mi_c, int s) { /* s = square size in px */
    if (mi_r >= G->mi_rows || mi_c >= G->mi_cols)
        return;
    const int q   = s / 4; /* mi units */
    int       opt = (int)rng_below(G->r, s == 64 ? 8 : 6);
    if (s == 64 && opt >= 6)
        opt = 3; /* SB64: split more often */
    if (s == 8 && opt >= 4)
        opt = (int)rng_below(G->r, 4);
    switch (opt) {
    case 0: place(G, mi_r, mi_c, s, s); break;
    case 1: place(G, mi_r, mi_c, s, s / 2), place(G, mi_r + q / 2, mi_c, s, s / 2); break;
    case 2: place(G, mi_r, mi_c, s / 2, s), place(G, mi_r, mi_c + q / 2, s / 2, s); break;
    case 3:
        if (s == 8)
            for (int k = 0; k < 4; k++) place(G, mi_r + (k >> 1), mi_c + (k & 1), 4, 4);
        else
            for (int k = 0; k < 4; k++) partition(G, mi_r + (k >> 1) * q / 2, mi_c + (k & 1) * q / 2, s / 2);
        break;
    case 4:
        for (int k = 0; k < 4; k++) place(G, mi_r + k * q / 4, mi_c, s, s / 4);
        break;
    default:
        for (int k = 0; k < 4; k++) place(G, mi_r, mi_c + k * q / 4, s / 4, s);
        break;
    }
}

static void fill_plane(Rng *r, uint16_t *p, int w, int h, int bd, int texture) {
    const int maxv = (1 << bd) - 1, one = 1 << (bd - 8);
    int       dc[64][64];
    for (int i = 0; i < 64; i++)
        for (int j = 0; j < 64; j++) dc[i][j] = ((int)rng_below(r, 2 * texture + 1) - texture) * one;
    const int base = (int)rng_below(r, (uint32_t)maxv / 2) + maxv / 4;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int v = base + (x * 2 + y) * one / 8 + dc[(y >> 3) & 63][(x >> 3) & 63];
            if (rng_below(r, 4) == 0)
                v += ((int)rng_below(r, 3) - 1) * one;
            p[y * w + x] = (uint16_t)clampi(v, 0, maxv);
        }
}

static void gen_frames(const char *dir) {
    static const FrameCase cases[] = {
        /* w    h  bd p16 ps pe  fl0 fl1 flu flv sh mrd seg */
        {64, 64, 8, 0, 0, 3, 32, 16, 10, 12, 0, 0, 0},
        {136, 72, 8, 0, 0, 3, 20, 24, 8, 0, 0, 1, 0},
        {200, 136, 10, 1, 0, 3, 32, 16, 16, 24, 0, 1, 1},
        {96, 80, 10, 1, 0, 3, 63, 40, 63, 5, 3, 0, 0},
        {128, 128, 8, 1, 0, 3, 12, 12, 30, 30, 6, 1, 1},
        {72, 40, 10, 1, 0, 3, 0, 0, 20, 20, 0, 0, 0},  /* luma off: the reference skips chroma too */
        {160, 96, 10, 1, 1, 3, 30, 30, 25, 0, 0, 1, 0}, /* chroma-only pass (level search trial) */
        {120, 64, 8, 0, 0, 1, 5, 50, 0, 0, 1, 0, 1},
        /* pictures off the 8-sample grid (coded size w x h, unpadded w - pad_right x h - pad_bottom, kPad): edges at
         * or past the unpadded size are not filtered (set_lpf_parameters, EbDeblockingFilter.c:173-178) */
        {200, 136, 10, 1, 0, 3, 40, 24, 20, 30, 0, 1, 0},
        {136, 72, 8, 0, 0, 3, 30, 36, 16, 12, 2, 0, 1},
        {96, 80, 10, 1, 0, 3, 63, 50, 40, 40, 0, 0, 0},
    };
    /* {pad_right, pad_bottom} of the cases above (0 before the crop cases) */
    static const int kPad[][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {6, 2}, {2, 6}, {4, 4}};
    const int ncase = (int)(sizeof(cases) / sizeof(cases[0]));
    char      path[512];
    snprintf(path, sizeof path, "%s/dlf_frame.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0xD1F0000000000002ull};
    uint32_t   nc = (uint32_t)ncase;
    golden_put1(&g, "ncase", 'I', 1, &nc);
    for (int ci = 0; ci < ncase; ci++) {
        const FrameCase *c = &cases[ci];
        const int        W = c->w, H = c->h, cw = W / 2, ch = H / 2;
        SequenceControlSet       *scs  = calloc(1, sizeof(*scs));
        PictureParentControlSet  *ppcs = calloc(1, sizeof(*ppcs));
        PictureControlSet        *pcs  = calloc(1, sizeof(*pcs));
        pcs->scs                       = scs;
        pcs->ppcs                      = ppcs;
        ppcs->scs                      = scs;
        scs->sb_size                   = 64;
        scs->seq_header.sb_size        = BLOCK_64X64;
        scs->is_16bit_pipeline         = (uint8_t)c->pipe16;
        scs->static_config.encoder_bit_depth = (uint32_t)c->bd;
        scs->max_input_luma_width      = (uint16_t)W;
        scs->max_input_luma_height     = (uint16_t)H;
        scs->max_input_pad_right       = (uint16_t)kPad[ci][0];
        scs->max_input_pad_bottom      = (uint16_t)kPad[ci][1];
        ppcs->aligned_width            = (uint16_t)W;
        ppcs->aligned_height           = (uint16_t)H;
        FrameHeader       *fh          = &ppcs->frm_hdr;
        struct LoopFilter *lf          = &fh->loop_filter_params;
        lf->filter_level[0]            = c->fl0;
        lf->filter_level[1]            = c->fl1;
        lf->filter_level_u             = c->flu;
        lf->filter_level_v             = c->flv;
        lf->sharpness_level            = c->sharp;
        lf->mode_ref_delta_enabled     = (uint8_t)c->mrd;
        static const int8_t def_ref[8] = {1, 0, 0, 0, -1, 0, -1, -1};
        for (int k = 0; k < 8; k++) lf->ref_deltas[k] = c->mrd == 1 && ci % 2 ? (int8_t)((int)rng_below(&r, 31) - 15) : def_ref[k];
        for (int k = 0; k < 2; k++) lf->mode_deltas[k] = c->mrd ? (int8_t)((int)rng_below(&r, 11) - 5) : 0;
        SegmentationParams *sp  = &fh->segmentation_params;
        sp->segmentation_enabled = (uint8_t)c->seg;
        if (c->seg)
            for (int s = 0; s < 8; s++)
                for (int f = 1; f <= 4; f++) {
                    sp->feature_enabled[s][f] = rng_below(&r, 2);
                    sp->feature_data[s][f]    = (int16_t)((int)rng_below(&r, 127) - 63);
                }
        /* mode info grid */
        const int mi_cols = ((W + 7) & ~7) >> 2, mi_rows = ((H + 7) & ~7) >> 2;
        Grid      G;
        G.cap     = mi_rows * mi_cols;
        G.blocks  = calloc((size_t)G.cap, sizeof(MbModeInfo));
        G.nblocks = 0;
        G.cells   = calloc((size_t)G.cap, sizeof(ModeInfo *));
        G.mi_rows = mi_rows;
        G.mi_cols = mi_cols;
        G.r       = &r;
        G.seg     = c->seg;
        for (int sr = 0; sr < mi_rows; sr += 16)
            for (int sc = 0; sc < mi_cols; sc += 16) partition(&G, sr, sc, 64);
        pcs->mi_grid_base = G.cells;
        pcs->mi_stride    = (uint16_t)mi_cols;
        /* picture */
        uint16_t *pl[3];
        const int pw[3] = {W, cw, cw}, ph[3] = {H, ch, ch};
        for (int p = 0; p < 3; p++) {
            pl[p] = malloc(sizeof(uint16_t) * pw[p] * ph[p]);
            fill_plane(&r, pl[p], pw[p], ph[p], c->bd, 1 + ci % 4);
        }
        uint32_t dims2[2];
        char     nm[64];
#define PUT_PLANE(tag, p)                                                                 \
    dims2[0] = (uint32_t)ph[p], dims2[1] = (uint32_t)pw[p];                              \
    snprintf(nm, sizeof nm, "c%d_%s%d", ci, tag, p);                                      \
    golden_put(&g, nm, 'H', 2, dims2, pl[p]);
        for (int p = 0; p < 3; p++) { PUT_PLANE("in", p) }
        EbPictureBufferDesc pic;
        memset(&pic, 0, sizeof(pic));
        pic.bit_depth = c->bd > 8 ? EB_TEN_BIT : EB_EIGHT_BIT;
        pic.stride_y  = (uint16_t)W;
        pic.stride_cb = pic.stride_cr = (uint16_t)cw;
        uint8_t *b8[3] = {NULL, NULL, NULL};
        if (c->pipe16) {
            pic.buffer_y  = (uint8_t *)pl[0];
            pic.buffer_cb = (uint8_t *)pl[1];
            pic.buffer_cr = (uint8_t *)pl[2];
        } else {
            for (int p = 0; p < 3; p++) {
                b8[p] = malloc((size_t)pw[p] * ph[p]);
                for (int k = 0; k < pw[p] * ph[p]; k++) b8[p][k] = (uint8_t)pl[p][k];
            }
            pic.buffer_y = b8[0], pic.buffer_cb = b8[1], pic.buffer_cr = b8[2];
        }
        svt_av1_loop_filter_init(pcs);
        svt_av1_loop_filter_frame(&pic, pcs, c->plane_start, c->plane_end);
        if (!c->pipe16)
            for (int p = 0; p < 3; p++) {
                for (int k = 0; k < pw[p] * ph[p]; k++) pl[p][k] = b8[p][k];
                free(b8[p]);
            }
        for (int p = 0; p < 3; p++) { PUT_PLANE("out", p) }
        /* parameters: {w, h, bd, pipe16, plane_start, plane_end, fl0, fl1, flu, flv, sharp, mrd, seg} +
         * ref_deltas[8] + mode_deltas[2] + seg feature enabled[8][8] + data[8][8] */
        int32_t prm[13 + 8 + 2 + 128];
        memcpy(prm, c, sizeof(FrameCase));
        for (int k = 0; k < 8; k++) prm[13 + k] = lf->ref_deltas[k];
        for (int k = 0; k < 2; k++) prm[21 + k] = lf->mode_deltas[k];
        for (int s = 0; s < 8; s++)
            for (int f = 0; f < 8; f++) {
                prm[23 + s * 8 + f]      = sp->feature_enabled[s][f];
                prm[23 + 64 + s * 8 + f] = sp->feature_data[s][f];
            }
        snprintf(nm, sizeof nm, "c%d_params", ci);
        golden_put1(&g, nm, 'i', (uint32_t)(sizeof(prm) / 4), prm);
        if (kPad[ci][0] || kPad[ci][1]) {
            const int32_t pad[2] = {kPad[ci][0], kPad[ci][1]};
            snprintf(nm, sizeof nm, "c%d_pad", ci);
            golden_put1(&g, nm, 'i', 2, pad);
        }
        /* mi grid as SvtGpuLfMi records {bsize, tx_depth, skip, ref_frame0, mode, segment_id, 0, 0} */
        uint8_t *mi = calloc((size_t)G.cap, 8);
        for (int k = 0; k < G.cap; k++) {
            const BlockModeInfoEnc *b = &((MbModeInfo *)G.cells[k])->block_mi;
            mi[8 * k + 0]             = (uint8_t)b->bsize;
            mi[8 * k + 1]             = b->tx_depth;
            mi[8 * k + 2]             = b->skip;
            mi[8 * k + 3]             = (uint8_t)(int8_t)b->ref_frame[0];
            mi[8 * k + 4]             = (uint8_t)b->mode;
            mi[8 * k + 5]             = b->segment_id;
        }
        uint32_t dm[3] = {(uint32_t)mi_rows, (uint32_t)mi_cols, 8};
        snprintf(nm, sizeof nm, "c%d_mi", ci);
        golden_put(&g, nm, 'B', 3, dm, mi);
        free(mi);
        for (int p = 0; p < 3; p++) free(pl[p]);
        free(G.blocks);
        free(G.cells);
        free(pcs);
        free(ppcs);
        free(scs);
    }
    golden_close(&g);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    bind_c_kernels();
    gen_lpf(argv[1]);
    gen_frames(argv[1]);
    printf("dlf golden vectors written to %s\n", argv[1]);
    return 0;
}
