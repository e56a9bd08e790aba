/*
 * dlf_oracle.c — CPU restatement of SVT-AV1 v2.1.0's deblocking loop filter (apply + level search).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Edge filters restate
 * Source/Lib/Common/Codec/EbDeblockingCommon.c; the frame driver restates
 * Source/Lib/Encoder/Codec/EbDeblockingFilter.c (set_lpf_parameters :162-282, filter_block_plane_vert/horz
 * :287-546, svt_aom_loop_filter_sb :547-622, svt_av1_loop_filter_frame :624-653, search_filter_level
 * :886-991, svt_av1_pick_filter_level :1129-1252) in the same SB-lagged order as the reference.
 * Pinned by tests/test_oracle_golden.py against vectors from the reference's own C.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))
#define CLAMP_(v, lo, hi) ((v) < (lo) ? (lo) : (v) > (hi) ? (hi) : (v))
#define RPOT(v, n) (((v) + ((1 << (n)) >> 1)) >> (n))

/* ------------------------------------------------------------------------------------------- */
/* Edge filters (one sample line across the edge).  px[] holds p6..p0 q0..q6 at indices 0..13.    */
/* With bd = 8 the highbd arithmetic equals the 8-bit int8 arithmetic of filter4/8/14.            */
/* ------------------------------------------------------------------------------------------- */
static int clamp_sc(int t, int bd) { /* signed_char_clamp(_high) (EbDeblockingCommon.c:26-35) */
    const int lo = -128 << (bd - 8), hi = (128 << (bd - 8)) - 1;
    return CLAMP_(t, lo, hi);
}

static void filter4_(int mask, int thresh, int *px, int bd) { /* filter4 / highbd_filter4 (:214-240, :436-468) */
    const int off = 0x80 << (bd - 8);
    const int t16 = thresh << (bd - 8);
    int      *op1 = &px[5], *op0 = &px[6], *oq0 = &px[7], *oq1 = &px[8];
    const int ps1 = *op1 - off, ps0 = *op0 - off, qs0 = *oq0 - off, qs1 = *oq1 - off;
    const int hev = (abs(*op1 - *op0) > t16 || abs(*oq1 - *oq0) > t16) ? -1 : 0;
    int       filter = clamp_sc(ps1 - qs1, bd) & hev;
    filter           = clamp_sc(filter + 3 * (qs0 - ps0), bd) & mask;
    const int f1     = clamp_sc(filter + 4, bd) >> 3;
    const int f2     = clamp_sc(filter + 3, bd) >> 3;
    *oq0             = clamp_sc(qs0 - f1, bd) + off;
    *op0             = clamp_sc(ps0 + f2, bd) + off;
    filter           = RPOT(f1, 1) & ~hev;
    *oq1             = clamp_sc(qs1 - filter, bd) + off;
    *op1             = clamp_sc(ps1 + filter, bd) + off;
}

/* filter length 4/6/8/14 on one line; thresholds as the reference's uint8 vectors' first byte */
static void lpf_line(int *px, int len, int blimit, int limit, int thresh, int bd) {
    const int lim = limit << (bd - 8), blim = blimit << (bd - 8), one = 1 << (bd - 8);
    const int p6 = px[0], p5 = px[1], p4 = px[2], p3 = px[3], p2 = px[4], p1 = px[5], p0 = px[6];
    const int q0 = px[7], q1 = px[8], q2 = px[9], q3 = px[10], q4 = px[11], q5 = px[12], q6 = px[13];
    const int edge = abs(p0 - q0) * 2 + abs(p1 - q1) / 2 > blim;
    if (len == 4) { /* filter_mask2 (:141-147) */
        const int m = !(abs(p1 - p0) > lim || abs(q1 - q0) > lim || edge) ? -1 : 0;
        filter4_(m, thresh, px, bd);
        return;
    }
    if (len == 6) { /* filter_mask3_chroma + flat_mask3_chroma + filter6 (:162-183, :274-287) */
        const int m = !(abs(p2 - p1) > lim || abs(p1 - p0) > lim || abs(q1 - q0) > lim || abs(q2 - q1) > lim || edge);
        const int flat = !(abs(p1 - p0) > one || abs(q1 - q0) > one || abs(p2 - p0) > one || abs(q2 - q0) > one);
        if (flat && m) {
            px[5] = RPOT(p2 * 3 + p1 * 2 + p0 * 2 + q0, 3);
            px[6] = RPOT(p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1, 3);
            px[7] = RPOT(p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2, 3);
            px[8] = RPOT(p0 + q0 * 2 + q1 * 2 + q2 * 3, 3);
        } else
            filter4_(m ? -1 : 0, thresh, px, bd);
        return;
    }
    /* filter_mask + flat_mask4 (:149-160, :196-206) */
    const int m = !(abs(p3 - p2) > lim || abs(p2 - p1) > lim || abs(p1 - p0) > lim || abs(q1 - q0) > lim ||
                    abs(q2 - q1) > lim || abs(q3 - q2) > lim || edge);
    const int flat = !(abs(p1 - p0) > one || abs(q1 - q0) > one || abs(p2 - p0) > one || abs(q2 - q0) > one ||
                       abs(p3 - p0) > one || abs(q3 - q0) > one);
    int flat2 = 0;
    if (len == 14) /* flat_mask4(1, p6, p5, p4, p0, q0, q4, q5, q6) (:806-807) */
        flat2 = !(abs(p5 - p0) > one || abs(q5 - q0) > one || abs(p4 - p0) > one || abs(q4 - q0) > one ||
                  abs(p6 - p0) > one || abs(q6 - q0) > one);
    if (len == 14 && flat2 && flat && m) { /* filter14 13-tap (:780-799) */
        px[1]  = RPOT(p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0, 4);
        px[2]  = RPOT(p6 * 5 + p5 * 2 + p4 * 2 + p3 * 2 + p2 + p1 + p0 + q0 + q1, 4);
        px[3]  = RPOT(p6 * 4 + p5 + p4 * 2 + p3 * 2 + p2 * 2 + p1 + p0 + q0 + q1 + q2, 4);
        px[4]  = RPOT(p6 * 3 + p5 + p4 + p3 * 2 + p2 * 2 + p1 * 2 + p0 + q0 + q1 + q2 + q3, 4);
        px[5]  = RPOT(p6 * 2 + p5 + p4 + p3 + p2 * 2 + p1 * 2 + p0 * 2 + q0 + q1 + q2 + q3 + q4, 4);
        px[6]  = RPOT(p6 + p5 + p4 + p3 + p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + q2 + q3 + q4 + q5, 4);
        px[7]  = RPOT(p5 + p4 + p3 + p2 + p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + q3 + q4 + q5 + q6, 4);
        px[8]  = RPOT(p4 + p3 + p2 + p1 + p0 + q0 * 2 + q1 * 2 + q2 * 2 + q3 + q4 + q5 + q6 * 2, 4);
        px[9]  = RPOT(p3 + p2 + p1 + p0 + q0 + q1 * 2 + q2 * 2 + q3 * 2 + q4 + q5 + q6 * 3, 4);
        px[10] = RPOT(p2 + p1 + p0 + q0 + q1 + q2 * 2 + q3 * 2 + q4 * 2 + q5 + q6 * 4, 4);
        px[11] = RPOT(p1 + p0 + q0 + q1 + q2 + q3 * 2 + q4 * 2 + q5 * 2 + q6 * 5, 4);
        px[12] = RPOT(p0 + q0 + q1 + q2 + q3 + q4 * 2 + q5 * 2 + q6 * 7, 4);
    } else if (flat && m) { /* filter8 7-tap (:289-304) */
        px[4] = RPOT(p3 + p3 + p3 + 2 * p2 + p1 + p0 + q0, 3);
        px[5] = RPOT(p3 + p3 + p2 + 2 * p1 + p0 + q0 + q1, 3);
        px[6] = RPOT(p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2, 3);
        px[7] = RPOT(p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3, 3);
        px[8] = RPOT(p1 + p0 + q0 + 2 * q1 + q2 + q3 + q3, 3);
        px[9] = RPOT(p0 + q0 + q1 + 2 * q2 + q3 + q3 + q3, 3);
    } else
        filter4_(m ? -1 : 0, thresh, px, bd);
}

/* one 4-sample edge segment; `step` = distance between samples across the edge, `adv` = along it */
#define DEFINE_LPF_SEG(NAME, T)                                                                              \
    static void NAME(T *s, long step, long adv, int len, int blimit, int limit, int thresh, int bd) {        \
        const int half = len == 14 ? 7 : len == 8 ? 4 : len == 6 ? 3 : 2;                                   \
        for (int i = 0; i < 4; i++, s += adv) {                                                              \
            int px[14] = {0};                                                                                \
            for (int k = -half; k < half; k++) px[7 + k] = s[k * step];                                      \
            lpf_line(px, len, blimit, limit, thresh, bd);                                                    \
            for (int k = -half; k < half; k++) s[k * step] = (T)px[7 + k];                                   \
        }                                                                                                    \
    }
DEFINE_LPF_SEG(lpf_seg8, uint8_t)
DEFINE_LPF_SEG(lpf_seg16, uint16_t)

void oracle_lpf(uint8_t *s, int32_t pitch, int vertical, int len, const uint8_t *blimit, const uint8_t *limit,
                const uint8_t *thresh) {
    lpf_seg8(s, vertical ? 1 : pitch, vertical ? pitch : 1, len, *blimit, *limit, *thresh, 8);
}
void oracle_highbd_lpf(uint16_t *s, int32_t pitch, int vertical, int len, const uint8_t *blimit, const uint8_t *limit,
                       const uint8_t *thresh, int32_t bd) {
    lpf_seg16(s, vertical ? 1 : pitch, vertical ? pitch : 1, len, *blimit, *limit, *thresh, bd);
}

/* ------------------------------------------------------------------------------------------- */
/* AV1 size tables (derived from the BlockSize / TxSize enums of EbDefinitions.h)                */
/* ------------------------------------------------------------------------------------------- */
/* BlockSize: 4X4 4X8 8X4 8X8 8X16 16X8 16X16 16X32 32X16 32X32 32X64 64X32 64X64 64X128 128X64 128X128
 *            4X16 16X4 8X32 32X8 16X64 64X16 */
static const int kBw[22] = {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 64, 128, 128, 4, 16, 8, 32, 16, 64};
static const int kBh[22] = {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 128, 64, 128, 16, 4, 32, 8, 64, 16};
/* TxSize: 4X4 8X8 16X16 32X32 64X64 4X8 8X4 8X16 16X8 16X32 32X16 32X64 64X32 4X16 16X4 8X32 32X8 16X64 64X16 */
static const int kTw[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
static const int kTh[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};

static int tx_of_dims(int w, int h) {
    for (int t = 0; t < 19; t++)
        if (kTw[t] == w && kTh[t] == h)
            return t;
    return -1;
}
static int bsize_of_dims(int w, int h) {
    for (int b = 0; b < 22; b++)
        if (kBw[b] == w && kBh[b] == h)
            return b;
    return -1;
}
/* tx_depth_to_tx_size (EbDefinitions.h:885-906), as TxSize indices (note 8X8 at depth 2 stays 8X8) */
static const int kTxDepth[3][22] = {{0, 5, 6, 1, 7, 8, 2, 9, 10, 3, 11, 12, 4, 4, 4, 4, 13, 14, 15, 16, 17, 18},
                                    {0, 5, 6, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 6, 7, 8, 9, 10},
                                    {0, 5, 6, 1, 0, 0, 0, 1, 1, 1, 2, 2, 2, 4, 4, 4, 0, 0, 1, 1, 2, 2}};
static int tx_for_depth(int bsize, int depth) { return kTxDepth[depth][bsize]; }
/* av1_get_max_uv_txsize for 4:2:0 (EbUtility.h:117-123): max transform of the subsampled block, 64s -> 32 */
static int uv_tx(int bsize) {
    int w = MAX_(kBw[bsize] >> 1, 4), h = MAX_(kBh[bsize] >> 1, 4);
    w = MIN_(w, 32);
    h = MIN_(h, 32);
    return tx_of_dims(w, h);
}
/* get_plane_block_size (ss_size_lookup[bsize][1][1]) for 4:2:0 */
static int uv_bsize(int bsize) { return bsize_of_dims(MAX_(kBw[bsize] >> 1, 4), MAX_(kBh[bsize] >> 1, 4)); }

static const int kModeLfLut[25] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, /* intra */
                                   1, 1, 0, 1,                            /* NEAREST NEAR GLOBAL NEW */
                                   1, 1, 1, 1, 1, 1, 0, 1};               /* compound; GLOBAL_GLOBAL 0 */

/* ------------------------------------------------------------------------------------------- */
/* Level tables: svt_av1_loop_filter_frame_init (EbDeblockingCommon.c:76-139),                    */
/* svt_aom_update_sharpness (:554-572), svt_av1_loop_filter_init (EbDeblockingFilter.c:35-47)     */
/* ------------------------------------------------------------------------------------------- */
typedef struct LfInfo {
    uint8_t mblim[64], lim[64], hev[64];
    uint8_t lvl[3][8][2][8][2];
} LfInfo;

static void lf_info_init(LfInfo *L, const SvtGpuLfParams *p, int plane_start, int plane_end) {
    const int sh = p->sharpness_level;
    for (int lvl = 0; lvl <= 63; lvl++) {
        int bil = lvl >> ((sh > 0) + (sh > 4));
        if (sh > 0 && bil > 9 - sh)
            bil = 9 - sh;
        if (bil < 1)
            bil = 1;
        L->lim[lvl]   = (uint8_t)bil;
        L->mblim[lvl] = (uint8_t)(2 * (lvl + 2) + bil);
        L->hev[lvl]   = (uint8_t)(lvl >> 4);
    }
    const int fl[3] = {p->filter_level[0], p->filter_level_u, p->filter_level_v};
    const int flr[3] = {p->filter_level[1], p->filter_level_u, p->filter_level_v};
    static const int seg_feat[3][2] = {{1, 2}, {3, 3}, {4, 4}}; /* seg_lvl_lf_lut */
    for (int plane = plane_start; plane < plane_end; plane++) {
        if (plane == 0 && !fl[0] && !flr[0])
            break;
        if ((plane == 1 && !fl[1]) || (plane == 2 && !fl[2]))
            continue;
        for (int seg = 0; seg < 8; seg++)
            for (int dir = 0; dir < 2; dir++) {
                int       lvl_seg = dir == 0 ? fl[plane] : flr[plane];
                const int f       = seg_feat[plane][dir];
                if (p->segmentation_enabled && p->seg_feature_enabled[seg][f])
                    lvl_seg = CLAMP_(lvl_seg + p->seg_feature_data[seg][f], 0, 63);
                if (!p->mode_ref_delta_enabled) {
                    memset(L->lvl[plane][seg][dir], lvl_seg, sizeof(L->lvl[plane][seg][dir]));
                } else {
                    const int scale = 1 << (lvl_seg >> 5);
                    L->lvl[plane][seg][dir][0][0] = (uint8_t)CLAMP_(lvl_seg + p->ref_deltas[0] * scale, 0, 63);
                    for (int ref = 1; ref < 8; ref++)
                        for (int mode = 0; mode < 2; mode++)
                            L->lvl[plane][seg][dir][ref][mode] =
                                (uint8_t)CLAMP_(lvl_seg + p->ref_deltas[ref] * scale + p->mode_deltas[mode] * scale, 0, 63);
                }
            }
    }
}

/* ------------------------------------------------------------------------------------------- */
/* Frame driver                                                                                  */
/* ------------------------------------------------------------------------------------------- */
typedef struct DlfCtx {
    const SvtGpuLfMi *mi;
    int               mi_rows, mi_cols;
    int               width, height; /* unpadded luma size (setup_dst_planes: frame width/height) */
    LfInfo            L;
    OracleFrame      *f;
} DlfCtx;

static int tx_dir(const SvtGpuLfMi *m, int vert, int plane, int skip) { /* get_transform_size (:143-160) */
    int ts = plane == 0 ? tx_for_depth(m->bsize, skip ? 0 : m->tx_depth) : uv_tx(m->bsize);
    /* txsize_horz_map / txsize_vert_map: the square transform of the extent across the edge */
    const int ext = vert ? kTw[ts] : kTh[ts];
    return tx_of_dims(ext, ext);
}

/* set_lpf_parameters (:162-282); returns the direction-mapped transform size, writes length/level */
static int lpf_params(const DlfCtx *C, int vert, int x, int y, int plane, int *len, int *level) {
    *len = 0;
    const int ss = plane ? 1 : 0;
    const int pw = plane ? C->width >> 1 : C->width, ph = plane ? C->height >> 1 : C->height;
    if (pw <= x || ph <= y)
        return 0; /* TX_4X4 */
    const int mi_row = ss | ((y << ss) >> 2), mi_col = ss | ((x << ss) >> 2);
    const SvtGpuLfMi *m = &C->mi[mi_row * C->mi_cols + mi_col];
    const int curr_skip = m->skip && m->ref_frame0 > 0;
    const int ts        = tx_dir(m, vert, plane, curr_skip);
    const int coord     = vert ? x : y;
    if (coord & (kTw[ts] - 1))
        return ts; /* not a transform edge */
    const int dir   = vert ? 0 : 1;
    const int curr  = C->L.lvl[plane][m->segment_id][dir][m->ref_frame0][kModeLfLut[m->mode]];
    int       lvl   = curr;
    if (coord) {
        const SvtGpuLfMi *pm = vert ? m - (1 << ss) : m - ((long)C->mi_cols << ss);
        const int pv_skip = pm->skip && pm->ref_frame0 > 0;
        const int pv_ts   = tx_dir(pm, vert, plane, pv_skip);
        const int pv_lvl  = C->L.lvl[plane][pm->segment_id][dir][pm->ref_frame0][kModeLfLut[pm->mode]];
        const int pb      = plane ? uv_bsize(m->bsize) : m->bsize;
        const int pu_edge = !(coord & ((vert ? kBw[pb] : kBh[pb]) - 1));
        if ((curr || pv_lvl) && (!pv_skip || !curr_skip || pu_edge)) {
            const int min_ts = MIN_(ts, pv_ts);
            *len             = min_ts == 0 ? 4 : plane ? 6 : (min_ts == 1 ? 8 : 14);
            lvl              = curr ? curr : pv_lvl;
        }
    }
    *level = lvl;
    return ts;
}

static void filter_at(const DlfCtx *C, int plane, int vert, int x, int y, int len, int lvl) {
    OracleFrame *f = C->f;
    const long   st = f->stride[plane];
    const int    bl = C->L.mblim[lvl], li = C->L.lim[lvl], th = C->L.hev[lvl];
    if (f->bit_depth > 8)
        lpf_seg16((uint16_t *)f->plane[plane] + (long)y * st + x, vert ? 1 : st, vert ? st : 1, len, bl, li, th,
                  f->bit_depth);
    else
        lpf_seg8((uint8_t *)f->plane[plane] + (long)y * st + x, vert ? 1 : st, vert ? st : 1, len, bl, li, th, 8);
}

/* svt_av1_filter_block_plane_vert / _horz (:287-546) for the SB at (mi_row, mi_col), SB64 */
static void filter_sb_plane(const DlfCtx *C, int plane, int vert, int mi_row, int mi_col) {
    const int ss = plane ? 1 : 0, range = 16 >> ss;
    for (int a = 0; a < range; a++) {        /* rows (vert) or columns (horz) of 4 samples */
        for (int b = 0; b < range;) {        /* along the filtering direction, stepping by transform size */
            const int cx = ((mi_col * 4) >> ss) + (vert ? b : a) * 4;
            const int cy = ((mi_row * 4) >> ss) + (vert ? a : b) * 4;
            int       len = 0, lvl = 0;
            const int ts = lpf_params(C, vert, cx, cy, plane, &len, &lvl);
            if (len)
                filter_at(C, plane, vert, cx, cy, len, lvl);
            b += (vert ? kTw[ts] : kTh[ts]) >> 2;
        }
    }
}

/* crop_w / crop_h: the unpadded size set_lpf_parameters stops at (scs->max_input_luma_width - max_input_pad_right,
 * EbDeblockingFilter.c:99-129); the frame is the coded size */
int oracle_dlf_frame_crop(OracleFrame *f, const SvtGpuLfMi *mi, const SvtGpuLfParams *p, int plane_start, int plane_end,
                          int crop_w, int crop_h) {
    DlfCtx C;
    C.mi      = mi;
    C.mi_cols = ((f->width + 7) & ~7) >> 2;
    C.mi_rows = ((f->height + 7) & ~7) >> 2;
    C.width   = crop_w;
    C.height  = crop_h;
    C.f       = f;
    lf_info_init(&C.L, p, plane_start, plane_end);
    const int nsb_c = (f->width + 63) / 64, nsb_r = (f->height + 63) / 64;
    const int fl[3] = {p->filter_level[0] | p->filter_level[1], p->filter_level_u, p->filter_level_v};
    /* svt_av1_loop_filter_frame (:624-653) → svt_aom_loop_filter_sb (:547-622), combine_vert_horz_lf */
    for (int r = 0; r < nsb_r; r++)
        for (int c = 0; c < nsb_c; c++)
            for (int plane = plane_start; plane < plane_end; plane++) {
                if (plane == 0 && !fl[0])
                    break; /* luma off stops all planes (:575-577) */
                if (!fl[plane])
                    continue;
                filter_sb_plane(&C, plane, 1, 16 * r, 16 * c);
                if (c > 0)
                    filter_sb_plane(&C, plane, 0, 16 * r, 16 * (c - 1));
                if (c == nsb_c - 1)
                    filter_sb_plane(&C, plane, 0, 16 * r, 16 * c);
            }
    return SVTGPU_OK;
}
int oracle_dlf_frame(OracleFrame *f, const SvtGpuLfMi *mi, const SvtGpuLfParams *p, int plane_start, int plane_end) {
    return oracle_dlf_frame_crop(f, mi, p, plane_start, plane_end, f->width, f->height);
}

/* ------------------------------------------------------------------------------------------- */
/* Level search (LPF_PICK_FROM_FULL_IMAGE)                                                       */
/* ------------------------------------------------------------------------------------------- */
static uint64_t plane_sse(const OracleFrame *a, const OracleFrame *b, int plane) {
    const int pw = plane ? a->width / 2 : a->width, ph = plane ? a->height / 2 : a->height;
    uint64_t  s  = 0;
    for (int r = 0; r < ph; r++)
        for (int c = 0; c < pw; c++) {
            const long ia = (long)r * a->stride[plane] + c, ib = (long)r * b->stride[plane] + c;
            const int  va = a->bit_depth > 8 ? ((uint16_t *)a->plane[plane])[ia] : ((uint8_t *)a->plane[plane])[ia];
            const int  vb = b->bit_depth > 8 ? ((uint16_t *)b->plane[plane])[ib] : ((uint8_t *)b->plane[plane])[ib];
            s += (uint64_t)((va - vb) * (va - vb));
        }
    return s;
}

static void copy_plane(OracleFrame *dst, const OracleFrame *src, int plane) {
    const int pw = plane ? src->width / 2 : src->width, ph = plane ? src->height / 2 : src->height;
    const int bps = src->bit_depth > 8 ? 2 : 1;
    for (int r = 0; r < ph; r++)
        memcpy((char *)dst->plane[plane] + (long)r * dst->stride[plane] * bps,
               (const char *)src->plane[plane] + (long)r * src->stride[plane] * bps, (size_t)pw * bps);
}

/* try_filter_frame (:841-883) */
static int64_t try_level(OracleFrame *recon, const OracleFrame *backup, const OracleFrame *src, const SvtGpuLfMi *mi,
                         SvtGpuLfParams *p, int lvl, int plane, int dir) {
    int fl[2] = {lvl, lvl};
    if (plane == 0 && dir == 0) fl[1] = p->filter_level[1];
    if (plane == 0 && dir == 1) fl[0] = p->filter_level[0];
    if (plane == 0) {
        p->filter_level[0] = fl[0];
        p->filter_level[1] = fl[1];
    } else if (plane == 1)
        p->filter_level_u = fl[0];
    else
        p->filter_level_v = fl[0];
    oracle_dlf_frame(recon, mi, p, plane, plane + 1);
    const int64_t e = (int64_t)plane_sse(src, recon, plane);
    copy_plane(recon, backup, plane);
    return e;
}

/* search_filter_level (:886-991) */
static int search_level(OracleFrame *recon, OracleFrame *backup, const OracleFrame *src, const SvtGpuLfMi *mi,
                        SvtGpuLfParams *p, const int last[4], int dlf_avg, int early_exit, int only4x4, int plane,
                        int dir) {
    int lvl = plane == 0 ? (dlf_avg ? last[0] : last[dir]) : last[plane + 1];
    int mid = CLAMP_(lvl, 0, 63), step = mid < 16 ? 4 : mid / 4, direction = 0;
    int64_t ss_err[64];
    for (int i = 0; i < 64; i++) ss_err[i] = -1;
    copy_plane(backup, recon, plane);
    int64_t best_err = try_level(recon, backup, src, mi, p, mid, plane, dir);
    int     best     = mid;
    ss_err[mid]      = best_err;
    int conv = 0;
    while (step > 0) {
        const int hi = MIN_(mid + step, 63), lo = MAX_(mid - step, 0);
        int64_t   bias = (best_err >> (15 - (mid / 8))) * step;
        if (!only4x4)
            bias >>= 1;
        if (direction <= 0 && lo != mid) {
            if (ss_err[lo] < 0)
                ss_err[lo] = try_level(recon, backup, src, mi, p, lo, plane, dir);
            if (ss_err[lo] < best_err + bias) {
                if (ss_err[lo] < best_err)
                    best_err = ss_err[lo];
                best = lo;
            }
        }
        if (direction >= 0 && hi != mid) {
            if (ss_err[hi] < 0)
                ss_err[hi] = try_level(recon, backup, src, mi, p, hi, plane, dir);
            if (ss_err[hi] < best_err - bias) {
                best_err = ss_err[hi];
                best     = hi;
            }
        }
        if (best == mid) {
            conv++;
            if (conv == early_exit)
                step = 0;
            else
                step /= 2;
            direction = 0;
        } else {
            direction = best < mid ? -1 : 1;
            mid       = best;
        }
    }
    return best;
}

/* svt_av1_pick_filter_level, FULL_IMAGE branch (:1146-1250) minus the reference-frame averaging
 * (the caller passes the averaged levels in `p` when dlf_avg is set). */
int oracle_dlf_pick(OracleFrame *recon, const OracleFrame *src, const SvtGpuLfMi *mi, SvtGpuLfParams *p, int dlf_avg,
                    int dlf_avg_uv, int temporal_layer_index, int early_exit, int only4x4) {
    OracleFrame backup = *recon;
    const int   bps    = recon->bit_depth > 8 ? 2 : 1;
    for (int pl = 0; pl < 3; pl++) {
        const int pw = pl ? recon->width / 2 : recon->width, ph = pl ? recon->height / 2 : recon->height;
        backup.plane[pl]  = malloc((size_t)pw * ph * bps);
        backup.stride[pl] = pw;
    }
    p->sharpness_level = 0;
    const int last[4]  = {p->filter_level[0], p->filter_level[1], p->filter_level_u, p->filter_level_v};
    const int y        = search_level(recon, &backup, src, mi, p, last, dlf_avg, early_exit, only4x4, 0, 2);
    p->filter_level[0] = p->filter_level[1] = y;
    if (dlf_avg_uv && temporal_layer_index > 0) {
        p->filter_level_u = last[2];
        p->filter_level_v = last[3];
    } else {
        p->filter_level_u = search_level(recon, &backup, src, mi, p, last, dlf_avg, early_exit, only4x4, 1, 0);
        p->filter_level_v = search_level(recon, &backup, src, mi, p, last, dlf_avg, early_exit, only4x4, 2, 0);
    }
    for (int pl = 0; pl < 3; pl++) free(backup.plane[pl]);
    return SVTGPU_OK;
}
