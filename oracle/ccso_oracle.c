/*
 * ccso_oracle.c — CPU restatement of CCSO, the fork's cross-component sample offset.
 * TEST INFRASTRUCTURE: imported only by tests/ (as the checker); never shipped or measured.
 * Pinned by tests/golden/ccso.bin (oracle/ref_harness/gen_golden_ccso.c: the reference's own EbCcso.c / EbPickccso.c
 * compiled from /root/reference by oracle/ref.mk).
 *
 * This is the reference's algorithm as written -- every configuration trained with a filtered copy of the plane and
 * a per-block SSD on every training pass -- not the device's moment formulation (csrc/ccso.hip), so the two are
 * independent derivations of the same numbers.
 *   oracle_ccso_extend        ext_rec_y: copy (EbPickccso.c:907-918) + extend_ccso_border (EbCcso.c:185-201)
 *   oracle_ccso_apply_plane   ccso_frame's body for one plane (EbCcso.c:637-677; the four apply functions :297-622,
 *                             ccso_filter_block_hbd_wo_buf_c :261-294, cal_filter_support :238-259)
 *   oracle_ccso_search_plane  derive_ccso_filter (EbPickccso.c:464-779) with compute_distortion (:55-68),
 *                             derive_blk_md (:71-120), ccso_derive_src_info (:125-160), the class-error passes
 *                             (:162-234, :382-428), the trial filters (:238-357), count_lut_bits (:360-378) and
 *                             derive_lut_offset (:431-461)
 *   oracle_ccso_search_frame  ccso_search (EbPickccso.c:785-815)
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/svtgpu.h"

#define PAD 5
#define BAND_NUM 128
#define MAX_ITER 15 /* CCSO_MAX_ITERATIONS (EbPickccso.h:7) */

static const int     kOffset[8]  = {-10, -7, -3, -1, 0, 1, 3, 7};  /* ccso_offset (EbPickccso.c:43) */
static const uint8_t kQuant[4]   = {16, 8, 32, 64};                /* quant_sz (EbPickccso.c:44, EbCcso.c:636) */
static const int     kEdgeInt[2] = {3, 2};                          /* edge_clf_to_edge_interval (EbCcso.h:22) */

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* derive_ccso_sample_pos (EbCcso.c:204-234) */
static void sample_pos(int *loc, int stride, int sup) {
    switch (sup) {
    case 0: loc[0] = -stride, loc[1] = stride; break;
    case 1: loc[0] = -stride - 1, loc[1] = stride + 1; break;
    case 2: loc[0] = -1, loc[1] = 1; break;
    case 3: loc[0] = stride - 1, loc[1] = -stride + 1; break;
    case 4: loc[0] = -3, loc[1] = 3; break;
    default: loc[0] = -5, loc[1] = 5; break;
    }
}

/* cal_filter_support (EbCcso.c:238-259) */
static void classify(int *cls, const uint16_t *p, int q, int nq, const int *loc, int edge_clf) {
    for (int i = 0; i < 2; i++) {
        const int d = p[loc[i]] - p[0];
        if (edge_clf == 0) cls[i] = d > q ? 2 : d < nq ? 0 : 1;
        else cls[i] = d < nq ? 0 : 1;
    }
}

/* grid of filter blocks on the 8-aligned mode-info grid (EbPickccso.c:473-476) */
static void grid(int w, int h, int plane, int *nvfb, int *nhfb) {
    const int ss = plane > 0, log2 = plane ? 7 : 8, unit = (1 << log2) >> 2;
    const int mi_rows = ((h + 7) & ~7) >> 2, mi_cols = ((w + 7) & ~7) >> 2;
    *nvfb = ((mi_rows >> ss) + unit - 1) / unit;
    *nhfb = ((mi_cols >> ss) + unit - 1) / unit;
}

int oracle_ccso_grid(int w, int h, int plane, int *nvfb, int *nhfb) {
    grid(w, h, plane, nvfb, nhfb);
    return 0;
}

void oracle_ccso_extend(const void *luma, int bits, int stride, int w, int h, uint16_t *ext) {
    const int es = w + 2 * PAD;
    for (int y = 0; y < h + 2 * PAD; y++)
        for (int x = 0; x < es; x++) {
            const int sy = clampi(y - PAD, 0, h - 1), sx = clampi(x - PAD, 0, w - 1);
            ext[(size_t)y * es + x] = bits == 8 ? ((const uint8_t *)luma)[(size_t)sy * stride + sx]
                                                : ((const uint16_t *)luma)[(size_t)sy * stride + sx];
        }
}

/* One plane of ccso_frame: the plane is read into 16 bits, filtered block by block where the block flag is set,
 * written back (EbCcso.c:639-677).  Samples are 8- or 16-bit (dst_bits); flags are nvfb x nhfb. */
void oracle_ccso_apply_plane(const uint16_t *ext, int w, int h, int bd, int plane, void *dst, int dst_bits,
                             int dst_stride, const SvtGpuCcsoParams *p, const uint8_t *flags) {
    if (!p->enable) return;
    const int ss = plane > 0, pw = plane ? w >> 1 : w, ph = plane ? h >> 1 : h, es = w + 2 * PAD;
    const int log2 = plane ? 7 : 8, bs = 1 << log2, max_val = (1 << bd) - 1;
    const int shift = bd - p->max_band_log2, q = kQuant[p->quant_idx], single = p->max_band_log2 == 0;
    int       nvfb, nhfb, loc[2];
    grid(w, h, plane, &nvfb, &nhfb);
    sample_pos(loc, es, p->ext_filter_support);
    const uint16_t *src = ext + PAD * es + PAD;
    for (int y = 0; y < ph; y += bs)
        for (int x = 0; x < pw; x += bs) {
            if (!flags[(y >> log2) * nhfb + (x >> log2)]) continue;
            const int y_end = ph - y < bs ? ph - y : bs, x_end = pw - x < bs ? pw - x : bs;
            for (int yy = y; yy < y + y_end; yy++)
                for (int xx = x; xx < x + x_end; xx++) {
                    const uint16_t *c = src + (size_t)(yy << ss) * es + (xx << ss);
                    int             cls[2] = {0, 0};
                    if (!p->bo_only) classify(cls, c, q, -q, loc, p->edge_clf);
                    const int band = single ? 0 : c[0] >> shift;
                    const int off  = p->filter_offset[(band << 4) + (cls[0] << 2) + cls[1]];
                    if (dst_bits == 8) {
                        uint8_t *d = (uint8_t *)dst + (size_t)yy * dst_stride + xx;
                        *d         = (uint8_t)clampi(off + *d, 0, max_val);
                    } else {
                        uint16_t *d = (uint16_t *)dst + (size_t)yy * dst_stride + xx;
                        *d          = (uint16_t)clampi(off + *d, 0, max_val);
                    }
                }
        }
}

/* ---- derive_ccso_filter ---- */
typedef struct {
    int      w, h, pw, ph, ss, log2, bs, nvfb, nhfb, nb;
    uint8_t *cls0, *cls1;                          /* at luma positions, stride w (ccso_stride) */
    int     *err[3][3][BAND_NUM], *cnt[3][3][BAND_NUM], *err_bo[BAND_NUM], *cnt_bo[BAND_NUM];
    uint32_t chroma_err[BAND_NUM * 16];             /* int in the reference; summed modulo 2^32 */
    int      chroma_cnt[BAND_NUM * 16];
} Search;

/* compute_distortion (EbPickccso.c:55-68) with compute_distortion_block_c (EbCcso.c:64-88) */
static uint64_t distortion(const Search *S, const uint16_t *org, const uint16_t *rec, uint64_t *buf) {
    uint64_t total = 0;
    for (int y = 0; y < S->ph; y += S->bs)
        for (int x = 0; x < S->pw; x += S->bs) {
            const int yo = y + S->bs >= S->ph ? S->ph - y : S->bs, xo = x + S->bs >= S->pw ? S->pw - x : S->bs;
            uint64_t  ssd = 0;
            for (int r = 0; r < yo; r++)
                for (int c = 0; c < xo; c++) {
                    const int e = org[(size_t)(y + r) * S->w + x + c] - rec[(size_t)(y + r) * S->w + x + c];
                    ssd += (uint64_t)(e * e);
                }
            buf[(y >> S->log2) * S->nhfb + (x >> S->log2)] = ssd;
            total += ssd;
        }
    return total;
}

/* RDCOST_DBL_WITH_NATIVE_BD_DIST1 (EbPickccso.h:9) over RDCOST_DBL (EbRestoration.h:346) */
static double rdcost(int rdmult, int bits, uint64_t dist, int bd) {
    const double d = (double)(dist >> (2 * (bd - 8)));
    return (((double)bits * rdmult) / (double)(1 << 9)) + (d * (1 << 7));
}

/* derive_lut_offset (EbPickccso.c:431-461); C float arithmetic as the reference evaluates it */
static void lut_offset(const Search *S, int8_t *lut, int band_log2, int edges) {
    for (int d0 = 0; d0 < edges; d0++)
        for (int d1 = 0; d1 < edges; d1++)
            for (int b = 0; b < (1 << band_log2); b++) {
                const int i = (b << 4) + (d0 << 2) + d1;
                if (!S->chroma_cnt[i]) continue;
                const float t = (float)(int32_t)S->chroma_err[i] / S->chroma_cnt[i];
                if (t < kOffset[0] || t >= kOffset[7]) {
                    lut[i] = (int8_t)clampi((int)t, kOffset[0], kOffset[7]);
                } else {
                    for (int k = 0; k < 7; k++)
                        if (t >= kOffset[k] && t <= kOffset[k + 1]) {
                            const float lo = t - kOffset[k], hi = t - kOffset[k + 1];
                            lut[i] = (int8_t)(fabs(lo) > fabs(hi) ? kOffset[k + 1] : kOffset[k]);
                            break;
                        }
                }
            }
}

/* count_lut_bits (EbPickccso.c:360-378) */
static int lut_bits(const int8_t *lut, int band_log2, int edges) {
    static const int reordered[8] = {0, 1, -1, 3, -3, 7, -7, -10};
    int              bits         = 0;
    for (int d0 = 0; d0 < edges; d0++)
        for (int d1 = 0; d1 < edges; d1++)
            for (int b = 0; b < (1 << band_log2); b++)
                for (int k = 0; k < 7; k++) {
                    bits++;
                    if (reordered[k] == lut[(b << 4) + (d0 << 2) + d1]) break;
                }
    return bits;
}

/* the trial filter of every block with the derived table (ccso_try_{luma,chroma}_filter, EbPickccso.c:238-357, over
 * ccso_filter_block_hbd_with_buf_c, EbCcso.c:6-37) */
static void trial_filter(const Search *S, const uint16_t *src, uint16_t *dst, const int8_t *lut, int shift, int bo,
                         int max_val) {
    for (int y = 0; y < S->ph; y++)
        for (int x = 0; x < S->pw; x++) {
            const size_t l  = (size_t)(y << S->ss) * S->w + (x << S->ss);
            const int    c0 = bo ? 0 : S->cls0[l], c1 = bo ? 0 : S->cls1[l];
            const int    band = src[(size_t)(y << S->ss) * (S->w + 2 * PAD) + (x << S->ss)] >> shift;
            uint16_t    *d    = dst + (size_t)y * S->w + x;
            *d                = (uint16_t)clampi(lut[(band << 4) + (c0 << 2) + c1] + *d, 0, max_val);
        }
}

static double search_plane(const uint16_t *ext, const uint16_t *org, const uint16_t *rec, int w, int h, int plane,
                           int bd, int rdmult, SvtGpuCcsoParams *out, uint8_t *flags_out) {
    Search S;
    memset(&S, 0, sizeof S);
    S.w = w, S.h = h, S.ss = plane > 0, S.pw = plane ? w >> 1 : w, S.ph = plane ? h >> 1 : h;
    S.log2 = plane ? 7 : 8, S.bs = 1 << S.log2;
    grid(w, h, plane, &S.nvfb, &S.nhfb);
    S.nb = S.nvfb * S.nhfb;
    const int es = w + 2 * PAD, nb = S.nb, max_val = (1 << bd) - 1;
    const uint16_t *src = ext + PAD * es + PAD;
    uint64_t *unf = calloc(nb, 8), *trn = calloc(nb, 8);
    uint8_t  *ctrl = calloc(nb, 1), *best_ctrl = calloc(nb, 1), *final_ctrl = calloc(nb, 1);
    uint16_t *tmp = malloc(sizeof(uint16_t) * (size_t)h * w);
    S.cls0 = calloc((size_t)h * w, 1), S.cls1 = calloc((size_t)h * w, 1);
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++)
            for (int k = 0; k < BAND_NUM; k++) S.err[a][b][k] = calloc(nb, 4), S.cnt[a][b][k] = calloc(nb, 4);
    for (int k = 0; k < BAND_NUM; k++) S.err_bo[k] = calloc(nb, 4), S.cnt_bo[k] = calloc(nb, 4);

    const uint64_t unf_frame = distortion(&S, org, rec, unf);
    const double   best_unf  = rdcost(rdmult, 1, unf_frame, bd);
    double         final_cost = DBL_MAX;
    int8_t         lut[BAND_NUM * 16], best_lut[BAND_NUM * 16], final_lut[BAND_NUM * 16];
    memset(best_lut, 0, sizeof best_lut), memset(final_lut, 0, sizeof final_lut);
    int best_clf = 0, final_clf = 0, final_q = 0, final_sup = 0, final_bo = 0, final_band = 0;
    const int frame_bits = 10, frame_bits_bo = 5; /* EbPickccso.c:530-542 with CONFIG_CCSO_SIGFIX */
    for (int bo = 0; bo < 2; bo++)
        for (int sup = 0; sup < (bo ? 1 : 6); sup++)
            for (int qi = 0; qi < (bo ? 1 : 4); qi++)
                for (int clf = 0; clf < (bo ? 1 : 2); clf++) {
                    const int edges = kEdgeInt[clf];
                    if (!bo) { /* ccso_derive_src_info (EbPickccso.c:125-160) */
                        int loc[2];
                        sample_pos(loc, es, sup);
                        for (int y = 0; y < S.ph; y++)
                            for (int x = 0; x < S.pw; x++) {
                                int          cls[2];
                                const size_t l = (size_t)(y << S.ss) * w + (x << S.ss);
                                classify(cls, src + (size_t)(y << S.ss) * es + (x << S.ss), kQuant[qi], -kQuant[qi],
                                         loc, clf);
                                S.cls0[l] = (uint8_t)cls[0], S.cls1[l] = (uint8_t)cls[1];
                            }
                    }
                    for (int band_log2 = 0; band_log2 < (bo ? 8 : 4); band_log2++) {
                        const int shift = bd - band_log2;
                        double    best_cost = DBL_MAX, prev_cost = DBL_MAX;
                        int       enable = 1, keep = 1, iter = 0;
                        memset(ctrl, 1, nb);
                        /* ccso_pre_compute_class_err(_bo) (EbPickccso.c:162-197, 382-428): blocks numbered in the
                         * order the plane is walked */
                        for (int a = 0; a < 3; a++)
                            for (int b = 0; b < 3; b++)
                                for (int k = 0; k < BAND_NUM; k++)
                                    memset(S.err[a][b][k], 0, 4 * nb), memset(S.cnt[a][b][k], 0, 4 * nb);
                        for (int k = 0; k < BAND_NUM; k++) memset(S.err_bo[k], 0, 4 * nb), memset(S.cnt_bo[k], 0, 4 * nb);
                        int fb = 0;
                        for (int y = 0; y < S.ph; y += S.bs)
                            for (int x = 0; x < S.pw; x += S.bs, fb++) {
                                const int y_end = S.ph - y < S.bs ? S.ph - y : S.bs;
                                const int x_end = S.pw - x < S.bs ? S.pw - x : S.bs;
                                for (int yy = y; yy < y + y_end; yy++)
                                    for (int xx = x; xx < x + x_end; xx++) {
                                        const int band = src[(size_t)(yy << S.ss) * es + (xx << S.ss)] >> shift;
                                        const int e    = org[(size_t)yy * w + xx] - rec[(size_t)yy * w + xx];
                                        if (bo) {
                                            S.err_bo[band][fb] += e, S.cnt_bo[band][fb]++;
                                        } else {
                                            const size_t l = (size_t)(yy << S.ss) * w + (xx << S.ss);
                                            S.err[S.cls0[l]][S.cls1[l]][band][fb] += e;
                                            S.cnt[S.cls0[l]][S.cls1[l]][band][fb]++;
                                        }
                                    }
                            }
                        while (keep) {
                            int improvement = 0;
                            if (enable) {
                                /* ccso_compute_class_err (EbPickccso.c:202-234) + derive_lut_offset */
                                memset(S.chroma_err, 0, sizeof S.chroma_err);
                                memset(S.chroma_cnt, 0, sizeof S.chroma_cnt);
                                memset(lut, 0, sizeof lut);
                                for (int f = 0; f < nb; f++) {
                                    if (!ctrl[f]) continue;
                                    if (bo) {
                                        for (int b = 0; b < (1 << band_log2); b++)
                                            S.chroma_err[b << 4] += (uint32_t)S.err_bo[b][f],
                                                S.chroma_cnt[b << 4] += S.cnt_bo[b][f];
                                    } else {
                                        for (int d0 = 0; d0 < edges; d0++)
                                            for (int d1 = 0; d1 < edges; d1++)
                                                for (int b = 0; b < (1 << band_log2); b++) {
                                                    const int i = (b << 4) + (d0 << 2) + d1;
                                                    S.chroma_err[i] += (uint32_t)S.err[d0][d1][b][f];
                                                    S.chroma_cnt[i] += S.cnt[d0][d1][b][f];
                                                }
                                    }
                                }
                                lut_offset(&S, lut, band_log2, bo ? 1 : edges);
                            }
                            memcpy(tmp, rec, sizeof(uint16_t) * (size_t)h * w);
                            trial_filter(&S, src, tmp, lut, shift, bo, max_val);
                            distortion(&S, org, tmp, trn);
                            /* derive_blk_md (EbPickccso.c:71-120): the per-block rate it accumulates from the adapted
                             * CDF is never read (cur_total_rate, :666-687), so the choice is the smaller SSD */
                            uint64_t dist = 0;
                            int      any  = 0;
                            if (enable)
                                for (int f = 0; f < nb; f++) {
                                    const int on = trn[f] < unf[f];
                                    ctrl[f]      = (uint8_t)on;
                                    dist += on ? trn[f] : unf[f];
                                    any |= on;
                                }
                            enable = any;
                            if (enable) {
                                const int bits = lut_bits(lut, band_log2, bo ? 1 : edges) +
                                    (bo ? frame_bits_bo : frame_bits) + nb;
                                const double cost = rdcost(rdmult, bits, dist, bd);
                                if (cost < prev_cost) prev_cost = cost, improvement = 1;
                                if (cost < best_cost) {
                                    best_cost = cost;
                                    memcpy(best_lut, lut, sizeof lut);
                                    best_clf = clf;
                                    memcpy(best_ctrl, ctrl, nb);
                                }
                            }
                            iter++;
                            if (!improvement || iter > MAX_ITER) keep = 0;
                        }
                        if (best_cost < final_cost) {
                            final_cost = best_cost, final_q = qi, final_sup = sup, final_bo = bo;
                            memcpy(final_lut, best_lut, sizeof best_lut);
                            final_band = band_log2, final_clf = best_clf;
                            memcpy(final_ctrl, best_ctrl, nb);
                        }
                    }
                }
    memset(out, 0, sizeof *out);
    if (best_unf < final_cost) {
        memset(flags_out, 0, nb);
    } else {
        out->enable = 1, out->bo_only = (uint8_t)final_bo, out->quant_idx = (uint8_t)final_q;
        out->ext_filter_support = (uint8_t)final_sup, out->max_band_log2 = (uint8_t)final_band;
        out->edge_clf = (uint8_t)final_clf;
        memcpy(out->filter_offset, final_lut, sizeof final_lut);
        memcpy(flags_out, final_ctrl, nb);
    }
    free(unf), free(trn), free(ctrl), free(best_ctrl), free(final_ctrl), free(tmp), free(S.cls0), free(S.cls1);
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++)
            for (int k = 0; k < BAND_NUM; k++) free(S.err[a][b][k]), free(S.cnt[a][b][k]);
    for (int k = 0; k < BAND_NUM; k++) free(S.err_bo[k]), free(S.cnt_bo[k]);
    return final_cost;
}

int oracle_ccso_search_plane(const uint16_t *ext, const uint16_t *org, const uint16_t *rec, int w, int h, int plane,
                             int bd, int rdmult, SvtGpuCcsoParams *out, uint8_t *flags_out) {
    search_plane(ext, org, rec, w, h, plane, bd, rdmult, out, flags_out);
    return out->enable;
}

/* ccso_search (EbPickccso.c:785-815): returns 1 when the weighted rdmult overflows (nothing searched) */
int oracle_ccso_search_frame(const uint16_t *ext, const uint16_t *const org[3], const uint16_t *const rec[3], int w,
                             int h, int bd, int rdmult, int base_q_idx, SvtGpuCcsoParams out[3],
                             uint8_t *const flags[3], int *frame_flag) {
    const int64_t r = (int64_t)rdmult * clampi(base_q_idx, 1, 63);
    if (r >= INT_MAX) return 1;
    *frame_flag = 0;
    for (int p = 0; p < 3; p++) *frame_flag |= oracle_ccso_search_plane(ext, org[p], rec[p], w, h, p, bd, (int)r,
                                                                         &out[p], flags[p]);
    return 0;
}
