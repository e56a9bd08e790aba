/*
 * lr_search_oracle.c — CPU restatement of SVT-AV1 v2.1.0's loop-restoration search (TEST INFRASTRUCTURE ONLY).
 *
 * Restates Source/Lib/Encoder/Codec/EbRestorationPick.c: sse_restoration_unit (:56), try_restoration_unit_seg
 * (:129, filtering without stripe boundaries: use_boundaries_in_rest_search = 0, EbEncHandle.c:4162), pixel
 * proj error (:167-320), finer_search_pixel_proj_error (:320-413), svt_get_proj_subspace_c (:417-500),
 * encode_xq (:502), apply_sgr (:522), search_selfguided_restoration (:550-651), count_*_bits (:655, :1008),
 * svt_av1_compute_stats(_highbd)_c (:671-757), linsolve_wiener / update_{a,b}_sep_sym /
 * wiener_decompose_sep_sym / compute_score / finalize_sym_filter (:766-1006), finer_tile_search_wiener_seg
 * (:1042-1146), search_* seg/finish/switchable (:1148-1460), rest_finish_search (:1555-1634); the rate
 * helpers of EbEntropyCoding.c:2876-3022; the controls of EncModeConfig.c:1329-1445.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))
#define CLAMP_(v, lo, hi) ((v) < (lo) ? (lo) : (v) > (hi) ? (hi) : (v))

#define PRJ_MIN0 (-(1 << 7) * 3 / 4)
#define PRJ_MAX0 (PRJ_MIN0 + (1 << 7) - 1)
#define PRJ_MIN1 (-(1 << 7) / 4)
#define PRJ_MAX1 (PRJ_MIN1 + (1 << 7) - 1)
#define TAP_SCALE ((int64_t)1 << 16)
#define FILT_STEP 128
static const int kTapMin[3] = {3 - 8, -7 - 16, 15 - 32}, kTapMax[3] = {3 - 1 + 8, -7 - 1 + 16, 15 - 1 + 32};
static const int kTapK[3] = {1, 2, 3};
static const int kSgrR[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                                 {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};

int oracle_lr_controls_for_level(int wn, int sg, SvtGpuLrSearchControls *c) {
    memset(c, 0, sizeof *c);
    switch (wn) {
    case 0: break;
    case 1: c->wn_enabled = 1, c->wn_use_chroma = 1, c->wn_filter_tap_lvl = 1, c->wn_use_refinement = 1; break;
    case 2:
        c->wn_enabled = 1, c->wn_use_chroma = 1, c->wn_filter_tap_lvl = 1, c->wn_use_refinement = 1;
        c->wn_max_one_refinement_step = 1;
        break;
    case 3:
        c->wn_enabled = 1, c->wn_use_chroma = 1, c->wn_filter_tap_lvl = 2, c->wn_use_refinement = 1;
        c->wn_max_one_refinement_step = 1;
        break;
    case 4: c->wn_enabled = 1, c->wn_use_chroma = 1, c->wn_filter_tap_lvl = 2, c->wn_max_one_refinement_step = 1; break;
    case 5: c->wn_enabled = 1, c->wn_filter_tap_lvl = 2, c->wn_max_one_refinement_step = 1; break;
    default: return SVTGPU_ERR_UNSUPPORTED; /* 6: use_prev_frame_coeffs needs the previous frame */
    }
    static const int t[4][9] = {/* use_chroma, start0, end0, inc0, start1, end1, inc1, refine0, refine1 */
                                {1, 0, 16, 1, 0, 16, 1, 1, 1},
                                {1, 0, 16, 1, 4, 5, 1, 1, 0},
                                {1, 0, 16, 8, 4, 5, 1, 1, 0},
                                {0, 0, 16, 8, 4, 5, 1, 1, 0}};
    if (sg < 0 || sg > 4) return SVTGPU_ERR_UNSUPPORTED;
    if (sg > 0) {
        const int *r      = t[sg - 1];
        c->sg_enabled     = 1;
        c->sg_use_chroma  = r[0];
        c->sg_start_ep[0] = r[1], c->sg_end_ep[0] = r[2], c->sg_ep_inc[0] = r[3];
        c->sg_start_ep[1] = r[4], c->sg_end_ep[1] = r[5], c->sg_ep_inc[1] = r[6];
        c->sg_refine[0] = r[7], c->sg_refine[1] = r[8];
    }
    return SVTGPU_OK;
}

/* ------------------------------------------------------------------------------------------- */
/* plane view with edge clamping (the search's dgd buffer is extended by svt_extend_frame)        */
/* ------------------------------------------------------------------------------------------- */
typedef struct Pl {
    const void *p;
    int         stride, w, h, hb;
} Pl;
static inline int at(const Pl *q, int y, int x) {
    y = CLAMP_(y, 0, q->h - 1);
    x = CLAMP_(x, 0, q->w - 1);
    return q->hb ? ((const uint16_t *)q->p)[(long)y * q->stride + x] : ((const uint8_t *)q->p)[(long)y * q->stride + x];
}

typedef struct Lim {
    int h_start, h_end, v_start, v_end;
} Lim;

static int64_t sse_unit(const Pl *a, const Pl *b, const Lim *l) {
    int64_t s = 0;
    for (int y = l->v_start; y < l->v_end; y++)
        for (int x = l->h_start; x < l->h_end; x++) {
            const int d = at(a, y, x) - at(b, y, x);
            s += d * d;
        }
    return s;
}

/* filtered unit (try_restoration_unit_seg without boundaries) -> SSE against src */
static int64_t try_unit(const Pl *dgd, const Pl *src, const Lim *l, const SvtGpuRestUnit *u, int bd) {
    const int uw = l->h_end - l->h_start, uh = l->v_end - l->v_start;
    const int vs = uw + 8;
    uint16_t *v  = malloc(sizeof(uint16_t) * (size_t)vs * (uh + 7));
    for (int r = -3; r < uh + 4; r++)
        for (int c = -3; c < uw + 5; c++) v[(r + 3) * vs + c + 3] = (uint16_t)at(dgd, l->v_start + r, l->h_start + c);
    uint16_t *o = malloc(sizeof(uint16_t) * (size_t)uw * uh);
    if (u->type == SVTGPU_RESTORE_WIENER) {
        int r0, r1;
        oracle_wiener_round(bd, &r0, &r1);
        oracle_wiener_convolve(v + 3 * vs + 3, vs, o, uw, u->hfilter, u->vfilter, uw, uh, r0, r1, bd);
    } else {
        /* per-pixel filter over the (unpartitioned) unit: row parity is relative to the unit start, which is
         * even like every stripe / PU start of the reference */
        for (int j = 0; j < uw; j += 64) {
            const int w = MIN_(64, uw - j);
            for (int i = 0; i < uh; i += 64) {
                const int h = MIN_(64, uh - i);
                oracle_sgr_apply(v + (3 + i) * vs + 3 + j, vs, w, h, u->ep, u->xqd, o + i * uw + j, uw, bd);
            }
        }
    }
    int64_t s = 0;
    for (int y = 0; y < uh; y++)
        for (int x = 0; x < uw; x++) {
            const int d = (int)o[y * uw + x] - at(src, l->v_start + y, l->h_start + x);
            s += d * d;
        }
    free(v);
    free(o);
    return s;
}

/* ------------------------------------------------------------------------------------------- */
/* rates                                                                                         */
/* ------------------------------------------------------------------------------------------- */
static int msb(unsigned v) { return 31 - __builtin_clz(v); }
static int count_quniform(int n, int v) {
    if (n <= 1) return 0;
    const int l = msb((unsigned)(n - 1)) + 1, m = (1 << l) - n;
    return v < m ? l - 1 : l;
}
static int count_subexpfin(int n, int k, int v) {
    int count = 0, i = 0, mk = 0;
    for (;;) {
        const int b = i ? k + i - 1 : k, a = 1 << b;
        if (n <= mk + 3 * a) {
            count += count_quniform(n - mk, v - mk);
            break;
        }
        const int t = v >= mk + a;
        count++;
        if (t) {
            i++;
            mk += a;
        } else {
            count += b;
            break;
        }
    }
    return count;
}
static int recenter_nonneg(int r, int v) { return v > (r << 1) ? v : v >= r ? (v - r) << 1 : ((r - v) << 1) - 1; }
static int refsubexpfin(int n, int k, int ref, int v) {
    /* arguments are uint16_t in the reference */
    n &= 0xFFFF, ref &= 0xFFFF, v &= 0xFFFF;
    const int rv = (ref << 1) <= n ? recenter_nonneg(ref, v) : recenter_nonneg(n - 1 - ref, n - 1 - v);
    return count_subexpfin(n, k, rv & 0xFFFF);
}
static int count_wiener_bits(int win, const SvtGpuRestUnit *w, const SvtGpuRestUnit *ref) {
    int bits = 0;
    for (int f = 0; f < 2; f++) {
        const int16_t *a = f ? w->hfilter : w->vfilter, *r = f ? ref->hfilter : ref->vfilter;
        for (int t = win == 7 ? 0 : 1; t < 3; t++)
            bits += refsubexpfin(kTapMax[t] - kTapMin[t] + 1, kTapK[t], r[t] - kTapMin[t], a[t] - kTapMin[t]);
    }
    return bits;
}
static int count_sgrproj_bits(const SvtGpuRestUnit *s, const SvtGpuRestUnit *ref) {
    int bits = 4;
    if (kSgrR[s->ep][0] > 0) bits += refsubexpfin(PRJ_MAX0 - PRJ_MIN0 + 1, 4, ref->xqd[0] - PRJ_MIN0, s->xqd[0] - PRJ_MIN0);
    if (kSgrR[s->ep][1] > 0) bits += refsubexpfin(PRJ_MAX1 - PRJ_MIN1 + 1, 4, ref->xqd[1] - PRJ_MIN1, s->xqd[1] - PRJ_MIN1);
    return bits;
}
static double rdcost(int rdmult, int64_t bits, int64_t sse) {
    return ((double)bits * rdmult) / (double)(1 << 9) + (double)sse * (1 << 7);
}

/* ------------------------------------------------------------------------------------------- */
/* self-guided search                                                                            */
/* ------------------------------------------------------------------------------------------- */
static int64_t proj_err(const Pl *src, const Pl *dgd, const Lim *l, const int32_t *f0, const int32_t *f1, int fs,
                        const int32_t *xqd, int ep) {
    int32_t xq[2];
    oracle_decode_xq(xqd, xq, ep);
    int64_t err = 0;
    for (int i = 0; i < l->v_end - l->v_start; i++)
        for (int j = 0; j < l->h_end - l->h_start; j++) {
            const int d = at(dgd, l->v_start + i, l->h_start + j), s = at(src, l->v_start + i, l->h_start + j);
            const int u = d << 4;
            int       v = 1 << 10;
            if (kSgrR[ep][0] > 0) v += xq[0] * (f0[i * fs + j] - u);
            if (kSgrR[ep][1] > 0) v += xq[1] * (f1[i * fs + j] - u);
            const int e = (kSgrR[ep][0] > 0 || kSgrR[ep][1] > 0) ? (v >> 11) + d - s : d - s;
            err += e * e;
        }
    return err;
}

static int64_t finer_proj(const Pl *src, const Pl *dgd, const Lim *l, const int32_t *f0, const int32_t *f1, int fs,
                          int32_t *xqd, int refine, int ep) {
    int64_t err = proj_err(src, dgd, l, f0, f1, fs, xqd, ep);
    if (!refine) return err;
    const int tmin[2] = {PRJ_MIN0, PRJ_MIN1}, tmax[2] = {PRJ_MAX0, PRJ_MAX1};
    const int start = 2;
    for (int s = start; s >= 1; s >>= 1)
        for (int p = 0; p < 2; p++) {
            if (kSgrR[ep][p] == 0) continue;
            int skip = 0;
            for (;;) {
                if (xqd[p] - s >= tmin[p]) {
                    xqd[p] -= s;
                    const int64_t e2 = proj_err(src, dgd, l, f0, f1, fs, xqd, ep);
                    if (e2 > err)
                        xqd[p] += s;
                    else {
                        err  = e2;
                        skip = 1;
                        if (s == start) continue;
                    }
                }
                break;
            }
            if (skip) break; /* note: leaves the p loop (the reference's `break`) */
            for (;;) {
                if (xqd[p] + s <= tmax[p]) {
                    xqd[p] += s;
                    const int64_t e2 = proj_err(src, dgd, l, f0, f1, fs, xqd, ep);
                    if (e2 > err)
                        xqd[p] -= s;
                    else {
                        err = e2;
                        if (s == start) continue;
                    }
                }
                break;
            }
        }
    return err;
}

/* svt_get_proj_subspace_c + encode_xq */
static void proj_subspace(const Pl *src, const Pl *dgd, const Lim *l, const int32_t *f0, const int32_t *f1, int fs,
                          int ep, int32_t *xqd) {
    double    H[2][2] = {{0, 0}, {0, 0}}, C[2] = {0, 0};
    const int w = l->h_end - l->h_start, h = l->v_end - l->v_start, size = w * h;
    int32_t   xq[2] = {0, 0};
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            const double u  = (double)(at(dgd, l->v_start + i, l->h_start + j) << 4);
            const double s  = (double)(at(src, l->v_start + i, l->h_start + j) << 4) - u;
            const double g1 = kSgrR[ep][0] > 0 ? (double)f0[i * fs + j] - u : 0;
            const double g2 = kSgrR[ep][1] > 0 ? (double)f1[i * fs + j] - u : 0;
            H[0][0] += g1 * g1;
            H[1][1] += g2 * g2;
            H[0][1] += g1 * g2;
            C[0] += g1 * s;
            C[1] += g2 * s;
        }
    H[0][0] /= size;
    H[0][1] /= size;
    H[1][1] /= size;
    H[1][0] = H[0][1];
    C[0] /= size;
    C[1] /= size;
    if (kSgrR[ep][0] == 0) {
        const double det = H[1][1];
        if (!(det < 1e-8)) xq[1] = (int32_t)rint(C[1] / det * (1 << 7));
    } else if (kSgrR[ep][1] == 0) {
        const double det = H[0][0];
        if (!(det < 1e-8)) xq[0] = (int32_t)rint(C[0] / det * (1 << 7));
    } else {
        const double det = H[0][0] * H[1][1] - H[0][1] * H[1][0];
        if (!(det < 1e-8)) {
            const double x0 = (H[1][1] * C[0] - H[0][1] * C[1]) / det;
            const double x1 = (H[0][0] * C[1] - H[1][0] * C[0]) / det;
            xq[0]           = (int32_t)rint(x0 * (1 << 7));
            xq[1]           = (int32_t)rint(x1 * (1 << 7));
        }
    }
    if (kSgrR[ep][0] == 0) {
        xqd[0] = 0;
        xqd[1] = CLAMP_((1 << 7) - xq[1], PRJ_MIN1, PRJ_MAX1);
    } else if (kSgrR[ep][1] == 0) {
        xqd[0] = CLAMP_(xq[0], PRJ_MIN0, PRJ_MAX0);
        xqd[1] = CLAMP_((1 << 7) - xqd[0], PRJ_MIN1, PRJ_MAX1);
    } else {
        xqd[0] = CLAMP_(xq[0], PRJ_MIN0, PRJ_MAX0);
        xqd[1] = CLAMP_((1 << 7) - xqd[0] - xq[1], PRJ_MIN1, PRJ_MAX1);
    }
}

static void search_sgr(const Pl *dgd, const Pl *src, const Lim *l, int bd, int start, int end, int inc, int refine,
                       SvtGpuRestUnit *out) {
    const int w = l->h_end - l->h_start, h = l->v_end - l->v_start, es = w + 6;
    int32_t  *d  = malloc(sizeof(int32_t) * (size_t)es * (h + 6));
    int32_t  *f0 = malloc(sizeof(int32_t) * (size_t)w * h), *f1 = malloc(sizeof(int32_t) * (size_t)w * h);
    for (int i = -3; i < h + 3; i++)
        for (int j = -3; j < w + 3; j++) d[(i + 3) * es + j + 3] = at(dgd, l->v_start + i, l->h_start + j);
    int64_t besterr = -1;
    int     bestep  = 0, bestxqd[2] = {0, 0};
    for (int ep = start; ep < end; ep += inc) {
        /* apply_sgr over PUs: the filter is per pixel on the clamped frame (row parity from even starts) */
        for (int i = 0; i < h; i += 64)
            for (int j = 0; j < w; j += 64)
                oracle_sgr_filter(d + (3 + i) * es + 3 + j, es, MIN_(64, w - j), MIN_(64, h - i), ep, bd,
                                  f0 + i * w + j, f1 + i * w + j, w);
        int32_t xqd[2];
        proj_subspace(src, dgd, l, f0, f1, w, ep, xqd);
        const int64_t err = finer_proj(src, dgd, l, f0, f1, w, xqd, refine, ep);
        if (besterr == -1 || err < besterr) {
            bestep = ep, besterr = err, bestxqd[0] = xqd[0], bestxqd[1] = xqd[1];
        }
    }
    memset(out, 0, sizeof *out);
    out->type   = SVTGPU_RESTORE_SGRPROJ;
    out->ep     = bestep;
    out->xqd[0] = bestxqd[0];
    out->xqd[1] = bestxqd[1];
    free(d);
    free(f0);
    free(f1);
}

/* ------------------------------------------------------------------------------------------- */
/* Wiener search                                                                                 */
/* ------------------------------------------------------------------------------------------- */
static void compute_stats(int win, const Pl *dgd, const Pl *src, const Lim *l, int bd, int64_t *M, int64_t *H);
/* exported for the golden test: stats of the w x h block at (4, 4) of [h+8][st] planes */
void oracle_compute_stats(int win, const uint16_t *dgd, const uint16_t *src, int st, int w, int h, int bd, int64_t *M,
                          int64_t *H) {
    const Pl  d = {dgd, st, st, h + 8, 1}, s = {src, st, st, h + 8, 1};
    const Lim l = {4, 4 + w, 4, 4 + h};
    compute_stats(win, &d, &s, &l, bd, M, H);
}
static void compute_stats(int win, const Pl *dgd, const Pl *src, const Lim *l, int bd, int64_t *M, int64_t *H) {
    const int win2 = win * win, half = win >> 1;
    uint64_t  sum = 0;
    for (int i = l->v_start; i < l->v_end; i++)
        for (int j = l->h_start; j < l->h_end; j++) sum += (uint64_t)at(dgd, i, j);
    const int avg = (int)(sum / (uint64_t)((l->v_end - l->v_start) * (l->h_end - l->h_start)));
    memset(M, 0, sizeof(int64_t) * win2);
    memset(H, 0, sizeof(int64_t) * win2 * win2);
    int y[49];
    for (int i = l->v_start; i < l->v_end; i++)
        for (int j = l->h_start; j < l->h_end; j++) {
            const int x   = at(src, i, j) - avg;
            int       idx = 0;
            for (int k = -half; k <= half; k++)
                for (int q = -half; q <= half; q++) y[idx++] = at(dgd, i + q, j + k) - avg;
            for (int k = 0; k < win2; k++) {
                M[k] += (int64_t)y[k] * x;
                for (int q = k; q < win2; q++) H[k * win2 + q] += (int64_t)y[k] * y[q];
            }
        }
    const int div = bd == 12 ? 16 : bd == 10 ? 4 : 1;
    for (int k = 0; k < win2; k++) {
        M[k] /= div;
        H[k * win2 + k] /= div;
        for (int q = k + 1; q < win2; q++) {
            H[k * win2 + q] /= div;
            H[q * win2 + k] = H[k * win2 + q];
        }
    }
}

static int wrap_index(int i, int win) { return i >= (win >> 1) + 1 ? win - 1 - i : i; }

static int linsolve(int n, int64_t *A, int stride, int64_t *b, int32_t *x) {
    for (int k = 0; k < n - 1; k++) {
        for (int i = n - 1; i > k; i--)
            if (llabs(A[(i - 1) * stride + k]) < llabs(A[i * stride + k])) {
                for (int j = 0; j < n; j++) {
                    const int64_t c         = A[i * stride + j];
                    A[i * stride + j]       = A[(i - 1) * stride + j];
                    A[(i - 1) * stride + j] = c;
                }
                const int64_t c = b[i];
                b[i]            = b[i - 1];
                b[i - 1]        = c;
            }
        for (int i = k; i < n - 1; i++) {
            if (A[k * stride + k] == 0) return 0;
            const int64_t c = A[(i + 1) * stride + k], cd = A[k * stride + k];
            for (int j = 0; j < n; j++) A[(i + 1) * stride + j] -= c / 256 * A[k * stride + j] / cd * 256;
            b[i + 1] -= c * b[k] / cd;
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        if (A[i * stride + i] == 0) return 0;
        int64_t c = 0;
        for (int j = i + 1; j <= n - 1; j++) c += A[i * stride + j] * x[j] / TAP_SCALE;
        x[i] = (int32_t)(TAP_SCALE * (b[i] - c) / A[i * stride + i]);
    }
    return 1;
}

/* update_a_sep_sym (which = 0: fix b, solve a) / update_b_sep_sym (which = 1) */
static void update_sep_sym(int which, int win, const int64_t *M, const int64_t *H, int32_t *a, int32_t *b) {
    const int win2 = win * win, h1 = (win >> 1) + 1;
    int64_t   A[4] = {0}, B[16] = {0};
    int32_t   S[7];
#define HC(r, c) H[((r) / win) * win * win2 + ((r) % win) * win + (c)] /* hc[r][c] */
    if (!which) {
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++) A[wrap_index(j, win)] += M[i * win + j] * b[i] / TAP_SCALE;
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++)
                for (int k = 0; k < win; k++)
                    for (int l = 0; l < win; l++)
                        B[wrap_index(l, win) * h1 + wrap_index(k, win)] +=
                            HC(j * win + i, k * win2 + l) * b[i] / TAP_SCALE * b[j] / TAP_SCALE;
    } else {
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++) A[wrap_index(i, win)] += M[i * win + j] * a[j] / TAP_SCALE;
        for (int i = 0; i < win; i++)
            for (int j = 0; j < win; j++)
                for (int k = 0; k < win; k++)
                    for (int l = 0; l < win; l++)
                        B[wrap_index(j, win) * h1 + wrap_index(i, win)] +=
                            HC(i * win + j, k * win2 + l) * a[k] / TAP_SCALE * a[l] / TAP_SCALE;
    }
#undef HC
    const int64_t ah = A[h1 - 1];
    for (int i = 0; i < h1 - 1; i++) A[i] -= ah * 2 + B[i * h1 + h1 - 1] - 2 * B[(h1 - 1) * h1 + (h1 - 1)];
    for (int i = 0; i < h1 - 1; i++)
        for (int j = 0; j < h1 - 1; j++)
            B[i * h1 + j] -= 2 * (B[i * h1 + (h1 - 1)] + B[(h1 - 1) * h1 + j] - 2 * B[(h1 - 1) * h1 + (h1 - 1)]);
    if (linsolve(h1 - 1, B, h1, A, S)) {
        S[h1 - 1] = (int32_t)TAP_SCALE;
        for (int i = h1; i < win; i++) {
            S[i] = S[win - 1 - i];
            S[h1 - 1] -= 2 * S[i];
        }
        memcpy(which ? b : a, S, win * sizeof(int32_t));
    }
}

/* hc[r][c] = H + (r / win) * win * win2 + (r % win) * win + c, as wiener_decompose_sep_sym builds it */
static void decompose(int win, const int64_t *M, const int64_t *H, int32_t *a, int32_t *b) {
    static const int init[7] = {3, -7, 15, 128 - 22, 15, -7, 3}; /* WIENER_FILT_TAP3_MIDV includes the step */
    const int        off     = (7 - win) >> 1;
    for (int i = 0; i < win; i++) a[i] = b[i] = (int32_t)(TAP_SCALE / FILT_STEP * init[i + off]);
    for (int iter = 1; iter < 5; iter++) {
        update_sep_sym(0, win, M, H, a, b);
        update_sep_sym(1, win, M, H, a, b);
    }
}

static int64_t compute_score(int win, const int64_t *M, const int64_t *H, const int16_t *vf, const int16_t *hf) {
    int32_t   ab[49];
    int16_t   a[7], b[7];
    const int off = (7 - win) >> 1, win2 = win * win;
    a[3] = b[3] = FILT_STEP;
    for (int i = 0; i < 3; i++) {
        a[i] = a[6 - i] = vf[i];
        b[i] = b[6 - i] = hf[i];
        a[3] -= 2 * a[i];
        b[3] -= 2 * b[i];
    }
    for (int k = 0; k < win; k++)
        for (int l = 0; l < win; l++) ab[k * win + l] = a[l + off] * b[k + off];
    int64_t P = 0, Q = 0;
    for (int k = 0; k < win2; k++) {
        P += ab[k] * M[k] / FILT_STEP / FILT_STEP;
        for (int l = 0; l < win2; l++)
            Q += ab[k] * H[k * win2 + l] * ab[l] / FILT_STEP / FILT_STEP / FILT_STEP / FILT_STEP;
    }
    const int64_t score = Q - 2 * P;
    const int64_t i_score = H[(win2 >> 1) * win2 + (win2 >> 1)] - 2 * M[win2 >> 1];
    return score - i_score;
}

static void finalize(int win, const int32_t *f, int16_t *fi) {
    for (int i = 0; i < (win >> 1); i++) {
        const int64_t dividend = (int64_t)f[i] * FILT_STEP, divisor = TAP_SCALE;
        fi[i] = (int16_t)(dividend < 0 ? (dividend - divisor / 2) / divisor : (dividend + divisor / 2) / divisor);
    }
    if (win == 7) {
        fi[0] = (int16_t)CLAMP_(fi[0], kTapMin[0], kTapMax[0]);
        fi[1] = (int16_t)CLAMP_(fi[1], kTapMin[1], kTapMax[1]);
        fi[2] = (int16_t)CLAMP_(fi[2], kTapMin[2], kTapMax[2]);
    } else {
        fi[2] = (int16_t)CLAMP_(fi[1], kTapMin[2], kTapMax[2]);
        fi[1] = (int16_t)CLAMP_(fi[0], kTapMin[1], kTapMax[1]);
        fi[0] = 0;
    }
    fi[6] = fi[0];
    fi[5] = fi[1];
    fi[4] = fi[2];
    fi[3] = (int16_t)(-2 * (fi[0] + fi[1] + fi[2]));
}

static int64_t finer_wiener(const Pl *dgd, const Pl *src, const Lim *l, SvtGpuRestUnit *u, int win, int bd,
                            const SvtGpuLrSearchControls *c) {
    int64_t err = try_unit(dgd, src, l, u, bd);
    if (!c->wn_use_refinement) return err;
    const int off = (7 - win) >> 1, start = 4, end = c->wn_max_one_refinement_step ? 4 : 1;
    const int cont = !c->wn_max_one_refinement_step;
    for (int s = start; s >= end; s >>= 1)
        for (int f = 0; f < 2; f++) { /* hfilter taps, then vfilter taps */
            int16_t *t = f ? u->vfilter : u->hfilter;
            for (int p = off; p < 3; p++) {
                int skip = 0;
                for (;;) {
                    if (t[p] - s >= kTapMin[p]) {
                        t[p] -= s, t[6 - p] -= s, t[3] += 2 * s;
                        const int64_t e2 = try_unit(dgd, src, l, u, bd);
                        if (e2 > err)
                            t[p] += s, t[6 - p] += s, t[3] -= 2 * s;
                        else {
                            err  = e2;
                            skip = 1;
                            if (s == start && cont) continue;
                        }
                    }
                    break;
                }
                if (skip) break;
                for (;;) {
                    if (t[p] + s <= kTapMax[p]) {
                        t[p] += s, t[6 - p] += s, t[3] -= 2 * s;
                        const int64_t e2 = try_unit(dgd, src, l, u, bd);
                        if (e2 > err)
                            t[p] -= s, t[6 - p] -= s, t[3] += 2 * s;
                        else {
                            err = e2;
                            if (s == start && cont) continue;
                        }
                    }
                    break;
                }
            }
        }
    return err;
}

/* ------------------------------------------------------------------------------------------- */
/* frame                                                                                         */
/* ------------------------------------------------------------------------------------------- */
/* RestUnitSearchInfo (EbRestoration.h:349-360) as rest_finish_search uses it */
typedef struct Rusi {
    int64_t        sse[3];
    SvtGpuRestUnit wiener, sgrproj;
    int            best[3]; /* best_rtype[RESTORE_WIENER - 1 .. RESTORE_SWITCHABLE - 1] */
} Rusi;

int oracle_lr_search_frame(const OracleFrame *recon, const OracleFrame *source, const int *unit_size,
                           const SvtGpuLrSearchControls *c, int *frame_type_out, SvtGpuRestUnit *const *units_out,
                           SvtGpuLrUnitSearch *const *search_out) {
    const int bd = recon->bit_depth, hb = bd > 8;
    const int plane_end = ((c->wn_enabled && c->wn_use_chroma) || (c->sg_enabled && c->sg_use_chroma)) ? 2 : 0;
    for (int p = 0; p < 3; p++) frame_type_out[p] = SVTGPU_RESTORE_NONE;
    Rusi *rusi = NULL; /* rest_finish_search's per-unit array, shared by the planes (luma's unit count) */
    for (int p = 0; p <= plane_end; p++) {
        const int W = p ? (recon->width + 1) >> 1 : recon->width, H = p ? (recon->height + 1) >> 1 : recon->height;
        const Pl  dgd = {recon->plane[p], recon->stride[p], W, H, hb}, src = {source->plane[p], source->stride[p], W, H, hb};
        const int usz = unit_size[p], hu = oracle_lr_units(usz, W), vu = oracle_lr_units(usz, H), n = hu * vu;
        const int ext = usz * 3 / 2, off = 8 >> (p > 0);
        SvtGpuLrUnitSearch *rs  = calloc((size_t)n, sizeof *rs);
        Lim                *lim = calloc((size_t)n, sizeof *lim);
        int                 ui  = 0;
        for (int y0 = 0; y0 < H;) { /* foreach_rest_unit_in_tile */
            const int uh = (H - y0 < ext) ? H - y0 : usz;
            int       vs = MAX_(0, y0 - off), ve = y0 + uh;
            if (ve < H) ve -= off;
            for (int x0 = 0; x0 < W;) {
                const int uw = (W - x0 < ext) ? W - x0 : usz;
                lim[ui]      = (Lim){x0, x0 + uw, vs, ve};
                ui++;
                x0 += uw;
            }
            y0 += uh;
        }
        const int win_l = c->wn_filter_tap_lvl == 1 ? 7 : c->wn_filter_tap_lvl == 2 ? 5 : 3;
        const int win   = p == 0 ? win_l : MIN_(win_l, 5);
        for (int u = 0; u < n; u++) { /* restoration_seg_search */
            SvtGpuLrUnitSearch *r = &rs[u];
            r->sse[0]             = sse_unit(&src, &dgd, &lim[u]);
            if (c->wn_enabled && (!p || c->wn_use_chroma)) {
                int64_t M[49], Hm[49 * 49];
                int32_t vfd[7], hfd[7];
                compute_stats(win, &dgd, &src, &lim[u], bd, M, Hm);
                decompose(win, M, Hm, vfd, hfd);
                SvtGpuRestUnit w;
                memset(&w, 0, sizeof w);
                w.type = SVTGPU_RESTORE_WIENER;
                finalize(win, vfd, w.vfilter);
                finalize(win, hfd, w.hfilter);
                if (compute_score(win, M, Hm, w.vfilter, w.hfilter) > 0)
                    r->sse[1] = INT64_MAX;
                else {
                    r->sse[1] = finer_wiener(&dgd, &src, &lim[u], &w, win, bd, c);
                    r->wiener = w;
                }
            } else
                r->sse[1] = INT64_MAX;
            if (c->sg_enabled && (!p || c->sg_use_chroma)) {
                const int q = p > 0;
                search_sgr(&dgd, &src, &lim[u], bd, c->sg_start_ep[q], c->sg_end_ep[q], c->sg_ep_inc[q],
                           c->sg_refine[q], &r->sgrproj);
                r->sse[2] = try_unit(&dgd, &src, &lim[u], &r->sgrproj, bd);
            }
        }
        /* rest_finish_search (EbRestorationPick.c:1555-1634).  Its RestUnitSearchInfo array is allocated once for
         * the frame (luma's unit count) and shared by the planes: each finish pass overwrites only what it computes,
         * so a chroma plane's switchable pass reads the luma plane's best_rtype / sse / wiener (or sgrproj) entries
         * for a restoration type that chroma does not search (search_switchable :1148-1200 reads rusi->best_rtype,
         * rusi->sse, rusi->wiener, rusi->sgrproj; copy_unit_info :1202-1209 copies them) */
        if (p == 0) rusi = calloc((size_t)n, sizeof *rusi);
        const int force_all = c->wn_enabled && c->sg_enabled;
        const int force     = c->wn_enabled ? (c->sg_enabled ? 4 : 1) : (c->sg_enabled ? 2 : 0);
        const int nrt       = n > 1 ? 4 : 3;
        double    best_cost = 0;
        int       best_type = 0;
        for (int r = 0; r < nrt; r++) {
            if (!force_all && r != 0 && r != force) continue;
            if (p && ((r == 1 && !c->wn_use_chroma) || (r == 2 && !c->sg_use_chroma))) continue;
            /* search_rest_type_finish: rsc_on_tile resets the reference parameters */
            SvtGpuRestUnit refw, refs;
            memset(&refw, 0, sizeof refw);
            memset(&refs, 0, sizeof refs);
            static const int16_t defw[7] = {3, -7, 15, -22, 15, -7, 3};
            for (int k = 0; k < 7; k++) refw.vfilter[k] = refw.hfilter[k] = defw[k];
            refs.xqd[0] = (PRJ_MIN0 + PRJ_MAX0) / 2;
            refs.xqd[1] = (PRJ_MIN1 + PRJ_MAX1) / 2;
            int64_t sse = 0, bits = 0;
            for (int u = 0; u < n; u++) {
                const SvtGpuLrUnitSearch *R = &rs[u];
                Rusi                     *Q = &rusi[u];
                if (r == 0) { /* search_norestore_finish */
                    Q->sse[0] = R->sse[0];
                    sse += Q->sse[0];
                } else if (r == 1) { /* search_wiener_finish */
                    const int64_t bn = c->wiener_restore_cost[0];
                    Q->sse[1]        = R->sse[1];
                    if (Q->sse[1] == INT64_MAX) {
                        bits += bn;
                        sse += Q->sse[0];
                        Q->best[0] = 0;
                        continue;
                    }
                    Q->wiener        = R->wiener;
                    const int64_t bw = c->wiener_restore_cost[1] + ((int64_t)count_wiener_bits(win, &Q->wiener, &refw) << 9);
                    const double  cn = rdcost(c->rdmult, bn >> 4, Q->sse[0]), cw = rdcost(c->rdmult, bw >> 4, Q->sse[1]);
                    const int     t  = cw < cn;
                    Q->best[0]       = t ? 1 : 0;
                    sse += Q->sse[t ? 1 : 0];
                    bits += t ? bw : bn;
                    if (t) refw = Q->wiener;
                } else if (r == 2) { /* search_sgrproj_finish */
                    Q->sse[2]        = R->sse[2];
                    Q->sgrproj       = R->sgrproj;
                    const int64_t bn = c->sgrproj_restore_cost[0];
                    const int64_t bs = c->sgrproj_restore_cost[1] + ((int64_t)count_sgrproj_bits(&Q->sgrproj, &refs) << 9);
                    const double  cn = rdcost(c->rdmult, bn >> 4, Q->sse[0]), cs = rdcost(c->rdmult, bs >> 4, Q->sse[2]);
                    const int     t  = cs < cn;
                    Q->best[1]       = t ? 2 : 0;
                    sse += Q->sse[t ? 2 : 0];
                    bits += t ? bs : bn;
                    if (t) refs = Q->sgrproj;
                } else { /* search_switchable */
                    double  bc = 0;
                    int64_t bb = 0;
                    int     bt = 0;
                    for (int t = 0; t < 3; t++) {
                        if (t > 0 && Q->best[t - 1] == 0) continue;
                        /* search_switchable sizes the Wiener rate by plane only (7 luma / 5 chroma taps) */
                        const int win_sw = p == 0 ? 7 : 5;
                        int64_t   cp     = t == 1 ? count_wiener_bits(win_sw, &Q->wiener, &refw)
                                         : t == 2 ? count_sgrproj_bits(&Q->sgrproj, &refs)
                                                  : 0;
                        const int64_t b = c->switchable_restore_cost[t] + (cp << 9);
                        const double  cost = rdcost(c->rdmult, b >> 4, Q->sse[t]);
                        if (t == 0 || cost < bc) bc = cost, bb = b, bt = t;
                    }
                    Q->best[2] = bt;
                    sse += Q->sse[bt];
                    bits += bb;
                    if (bt == 1) refw = Q->wiener;
                    if (bt == 2) refs = Q->sgrproj;
                }
            }
            const double cost = rdcost(c->rdmult, bits >> 4, sse);
            if (r == 0 || cost < best_cost) best_cost = cost, best_type = r;
        }
        frame_type_out[p] = best_type;
        for (int u = 0; u < n; u++) { /* copy_unit_info */
            SvtGpuRestUnit o;
            memset(&o, 0, sizeof o);
            if (best_type != 0) {
                const int t = rusi[u].best[best_type - 1];
                o           = t == 1 ? rusi[u].wiener : rusi[u].sgrproj;
                o.type      = t;
            }
            if (units_out && units_out[p]) units_out[p][u] = o;
            if (search_out && search_out[p]) search_out[p][u] = rs[u];
        }
        free(rs);
        free(lim);
    }
    free(rusi);
    return SVTGPU_OK;
}

/* debug/test hook: the Wiener solve of one (M, H) */
void oracle_lr_debug_decompose(int win, const int64_t *M, const int64_t *H, int32_t *a, int32_t *b, int16_t *vf,
                               int16_t *hf, int64_t *score) {
    decompose(win, M, H, a, b);
    finalize(win, a, vf);
    finalize(win, b, hf);
    *score = compute_score(win, M, H, vf, hf);
}
void oracle_lr_debug_update(int which, int win, const int64_t *M, const int64_t *H, int32_t *a, int32_t *b) {
    update_sep_sym(which, win, M, H, a, b);
}

/* ------------------------------------------------------------------------------------------- */
/* measurement probe (not part of the restatement): for every unit of one plane and every ep of the search, the
 * exact error search_sgr finds (proj_subspace + finer_proj, EbRestorationPick.c:550-652) and a lower bound valid for
 * any xq: err >= (max(0, sqrt(Qmin) - sqrt(N) / 2))^2, Qmin the real least-squares minimum of the projection
 * residual over the unit (proj_err's per-pixel rounding moves each residual by at most 1/2).  Used to estimate how
 * many eps a bound-ordered search could skip (scripts/r5/sgr_prune_probe.py).  err/bound: [units][eps] */
int oracle_lr_sgr_probe(const uint16_t *dgd_p, int dgd_stride, const uint16_t *src_p, int src_stride, int W, int H,
                        int bd, int usz, int start, int end, int inc, int refine, int64_t *err_out, double *bound_out) {
    const Pl  dgd = {dgd_p, dgd_stride, W, H, 1}, src = {src_p, src_stride, W, H, 1};
    const int ext = usz * 3 / 2, off = 8;
    int       ui = 0, neps = 0;
    for (int ep = start; ep < end; ep += inc) neps++;
    for (int y0 = 0; y0 < H;) {
        const int uh = (H - y0 < ext) ? H - y0 : usz;
        int       vs = MAX_(0, y0 - off), ve = y0 + uh;
        if (ve < H) ve -= off;
        for (int x0 = 0; x0 < W;) {
            const int uw = (W - x0 < ext) ? W - x0 : usz;
            const Lim l  = {x0, x0 + uw, vs, ve};
            const int w = uw, h = ve - vs, es = w + 6;
            int32_t  *d  = malloc(sizeof(int32_t) * (size_t)es * (h + 6));
            int32_t  *f0 = malloc(sizeof(int32_t) * (size_t)w * h), *f1 = malloc(sizeof(int32_t) * (size_t)w * h);
            for (int i = -3; i < h + 3; i++)
                for (int j = -3; j < w + 3; j++) d[(i + 3) * es + j + 3] = at(&dgd, l.v_start + i, l.h_start + j);
            int k = 0;
            for (int ep = start; ep < end; ep += inc, k++) {
                for (int i = 0; i < h; i += 64)
                    for (int j = 0; j < w; j += 64)
                        oracle_sgr_filter(d + (3 + i) * es + 3 + j, es, MIN_(64, w - j), MIN_(64, h - i), ep, bd,
                                          f0 + i * w + j, f1 + i * w + j, w);
                int32_t xqd[2];
                proj_subspace(&src, &dgd, &l, f0, f1, w, ep, xqd);
                err_out[(size_t)ui * neps + k] = finer_proj(&src, &dgd, &l, f0, f1, w, xqd, refine, ep);
                double G00 = 0, G01 = 0, G11 = 0, c0 = 0, c1 = 0, yy = 0;
                for (int i = 0; i < h; i++)
                    for (int j = 0; j < w; j++) {
                        const int    dv = at(&dgd, vs + i, x0 + j), sv = at(&src, vs + i, x0 + j), u = dv << 4;
                        const double y  = (double)(sv - dv);
                        const double g0 = kSgrR[ep][0] > 0 ? (double)(f0[i * w + j] - u) : 0;
                        const double g1 = kSgrR[ep][1] > 0 ? (double)(f1[i * w + j] - u) : 0;
                        G00 += g0 * g0, G01 += g0 * g1, G11 += g1 * g1, c0 += g0 * y, c1 += g1 * y, yy += y * y;
                    }
                double       q   = yy;
                const double det = G00 * G11 - G01 * G01;
                if (det > 1e-9 * (G00 * G11 + 1))
                    q = yy - (G11 * c0 * c0 - 2 * G01 * c0 * c1 + G00 * c1 * c1) / det;
                else if (G00 > 0)
                    q = yy - c0 * c0 / G00;
                else if (G11 > 0)
                    q = yy - c1 * c1 / G11;
                const double r = sqrt(q > 0 ? q : 0) - sqrt((double)(w * h)) / 2;
                bound_out[(size_t)ui * neps + k] = r > 0 ? r * r : 0;
            }
            free(d), free(f0), free(f1);
            ui++;
            x0 += uw;
        }
        y0 += uh;
    }
    return ui;
}
