/*
 * lr_oracle.c — CPU restatement of SVT-AV1 v2.1.0's loop restoration (apply; search in lr_search_oracle.c).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Restates (paths under Source/Lib/):
 *   Common/Codec/convolve.c:109-232        Wiener convolve (add src), 8-bit and highbd
 *   Common/Codec/EbRestoration.c:466-955   box sums, self-guided filters (r = 2 "fast" on odd rows, r = 1)
 *   Common/Codec/EbRestoration.c:634-646, 957-991  decode_xq, apply_selfguided_restoration
 *   Common/Codec/EbRestoration.c:222-435, 1067-1139, 1179-1296  stripes, boundary substitution, units
 *   Common/Codec/EbRestoration.c:1522-1680 saved stripe boundary lines (deblocked / CDEF)
 * Pinned by tests/test_oracle_golden.py against tests/golden/lr_*.bin (reference C outputs).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))
#define CLAMP_(v, lo, hi) ((v) < (lo) ? (lo) : (v) > (hi) ? (hi) : (v))
#define RPOT(v, n) (((v) + ((1 << (n)) >> 1)) >> (n))

static const int kSgrR[16][2] = {{2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1}, {2, 1},
                                 {2, 1}, {2, 1}, {0, 1}, {0, 1}, {0, 1}, {0, 1}, {2, 0}, {2, 0}};
static const int kSgrS[16][2] = {{140, 3236}, {112, 2158}, {93, 1618}, {80, 1438}, {70, 1295}, {58, 1177},
                                 {47, 1079},  {37, 996},   {30, 925},  {25, 863},  {-1, 2589}, {-1, 1618},
                                 {-1, 1177},  {-1, 925},   {56, -1},   {22, -1}};
static const int kXByXPlus1[256] = {
    1,   128, 171, 192, 205, 213, 219, 224, 228, 230, 233, 235, 236, 238, 239, 240, 241, 242, 243, 243, 244, 244,
    245, 245, 246, 246, 247, 247, 247, 247, 248, 248, 248, 248, 249, 249, 249, 249, 249, 250, 250, 250, 250, 250,
    250, 250, 251, 251, 251, 251, 251, 251, 251, 251, 251, 251, 252, 252, 252, 252, 252, 252, 252, 252, 252, 252,
    252, 252, 252, 252, 252, 252, 252, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253,
    253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 253, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254,
    254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
    255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 256};
static const int kOneByX[25] = {4096, 2048, 1365, 1024, 819, 683, 585, 512, 455, 410, 372, 341, 315,
                                293,  273,  256,  241,  228, 216, 205, 195, 186, 178, 171, 164};

/* ------------------------------------------------------------------------------------------- */
/* Wiener convolve (add src): src points at output (0,0) of a buffer readable at rows -3..h+3,  */
/* cols -3..w+4; round0/round1 from get_conv_params_wiener (EbRestoration.c:49-72)              */
/* ------------------------------------------------------------------------------------------- */
void oracle_wiener_convolve(const uint16_t *src, int sstride, uint16_t *dst, int dstride, const int16_t *fx,
                            const int16_t *fy, int w, int h, int round0, int round1, int bd) {
    const int ih   = h + 7;
    uint16_t *temp = malloc(sizeof(uint16_t) * (size_t)ih * w);
    const int lim  = 1 << (bd + 1 + 7 - round0); /* WIENER_CLAMP_LIMIT */
    for (int y = 0; y < ih; y++)
        for (int x = 0; x < w; x++) {
            const uint16_t *s   = src + (long)(y - 3) * sstride + x - 3;
            int32_t         sum = ((int32_t)s[3] << 7) + (1 << (bd + 7 - 1));
            for (int k = 0; k < 8; k++) sum += s[k] * fx[k];
            temp[y * w + x] = (uint16_t)CLAMP_(RPOT(sum, round0), 0, lim - 1);
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const uint16_t *t   = temp + (long)y * w + x;
            int32_t         sum = ((int32_t)t[3 * w] << 7) - (1 << (bd + round1 - 1));
            for (int k = 0; k < 8; k++) sum += t[k * w] * fy[k];
            dst[(long)y * dstride + x] = (uint16_t)CLAMP_(RPOT(sum, round1), 0, (1 << bd) - 1);
        }
    free(temp);
}

void oracle_wiener_round(int bd, int *round0, int *round1) {
    *round0        = 3;
    *round1        = 2 * 7 - 3;
    const int over = bd + 7 - 3 + 2 - 16;
    if (over > 0) {
        *round0 += over;
        *round1 -= over;
    }
}

/* ------------------------------------------------------------------------------------------- */
/* self-guided filter                                                                           */
/* ------------------------------------------------------------------------------------------- */
/* full (2r+1)^2 box sum of x (sqr = 0) or x^2 at (i, j) of the int32 image d (valid for the A/B
 * positions the reference uses, which are >= 2 samples inside its extended box-sum region) */
static int32_t box(const int32_t *d, int stride, int i, int j, int r, int sqr) {
    int32_t s = 0;
    for (int y = -r; y <= r; y++)
        for (int x = -r; x <= r; x++) {
            const int32_t v = d[(long)(i + y) * stride + j + x];
            s += sqr ? v * v : v;
        }
    return s;
}

static void sgr_ab(const int32_t *dgd, int stride, int i, int j, int r, int s, int bd, int32_t *A, int32_t *B) {
    const int32_t n  = (2 * r + 1) * (2 * r + 1);
    const uint32_t a = (uint32_t)RPOT(box(dgd, stride, i, j, r, 1), 2 * (bd - 8));
    const uint32_t b = (uint32_t)RPOT(box(dgd, stride, i, j, r, 0), bd - 8);
    const uint32_t p = (a * n < b * b) ? 0 : a * n - b * b;
    const uint32_t z = (p * (uint32_t)s + (1u << 19)) >> 20; /* ROUND_POWER_OF_TWO(p * s, 20), uint32 */
    *A               = kXByXPlus1[MIN_(z, 255)];
    *B = (int32_t)(((uint32_t)(256 - *A) * (uint32_t)box(dgd, stride, i, j, r, 0) * (uint32_t)kOneByX[n - 1] +
                    (1u << 11)) >> 12);
}

/* dgd: int32 image readable at rows -3..h+2, cols -3..w+2 */
void oracle_sgr_filter(const int32_t *dgd, int stride, int w, int h, int eps, int bd, int32_t *flt0, int32_t *flt1,
                       int fstride) {
    const int bw = w + 2, bh = h + 2; /* A/B over [-1, h] x [-1, w] */
    int32_t  *A  = malloc(sizeof(int32_t) * bw * bh), *B = malloc(sizeof(int32_t) * bw * bh);
#define AB(arr, i, j) arr[((i) + 1) * bw + (j) + 1]
    if (kSgrR[eps][0] > 0) { /* selfguided_restoration_fast_internal, r = 2, A/B on odd rows */
        for (int i = -1; i < h + 1; i += 2)
            for (int j = -1; j < w + 1; j++)
                sgr_ab(dgd, stride, i, j, 2, kSgrS[eps][0], bd, &AB(A, i, j), &AB(B, i, j));
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++) {
                const int32_t x = dgd[(long)i * stride + j];
                int32_t       a, b, nb;
                if (!(i & 1)) {
                    a  = (AB(A, i - 1, j) + AB(A, i + 1, j)) * 6 +
                        (AB(A, i - 1, j - 1) + AB(A, i + 1, j - 1) + AB(A, i - 1, j + 1) + AB(A, i + 1, j + 1)) * 5;
                    b  = (AB(B, i - 1, j) + AB(B, i + 1, j)) * 6 +
                        (AB(B, i - 1, j - 1) + AB(B, i + 1, j - 1) + AB(B, i - 1, j + 1) + AB(B, i + 1, j + 1)) * 5;
                    nb = 5;
                } else {
                    a  = AB(A, i, j) * 6 + (AB(A, i, j - 1) + AB(A, i, j + 1)) * 5;
                    b  = AB(B, i, j) * 6 + (AB(B, i, j - 1) + AB(B, i, j + 1)) * 5;
                    nb = 4;
                }
                const int sh = 8 + nb - 4;
                flt0[(long)i * fstride + j] = (a * x + b + (1 << (sh - 1))) >> sh;
            }
    }
    if (kSgrR[eps][1] > 0) { /* selfguided_restoration_internal, r = 1, every row */
        for (int i = -1; i < h + 1; i++)
            for (int j = -1; j < w + 1; j++)
                sgr_ab(dgd, stride, i, j, 1, kSgrS[eps][1], bd, &AB(A, i, j), &AB(B, i, j));
        for (int i = 0; i < h; i++)
            for (int j = 0; j < w; j++) {
                const int32_t x = dgd[(long)i * stride + j];
                const int32_t a = (AB(A, i, j) + AB(A, i, j - 1) + AB(A, i, j + 1) + AB(A, i - 1, j) + AB(A, i + 1, j)) * 4 +
                    (AB(A, i - 1, j - 1) + AB(A, i + 1, j - 1) + AB(A, i - 1, j + 1) + AB(A, i + 1, j + 1)) * 3;
                const int32_t b = (AB(B, i, j) + AB(B, i, j - 1) + AB(B, i, j + 1) + AB(B, i - 1, j) + AB(B, i + 1, j)) * 4 +
                    (AB(B, i - 1, j - 1) + AB(B, i + 1, j - 1) + AB(B, i - 1, j + 1) + AB(B, i + 1, j + 1)) * 3;
                const int sh = 8 + 5 - 4;
                flt1[(long)i * fstride + j] = (a * x + b + (1 << (sh - 1))) >> sh;
            }
    }
#undef AB
    free(A);
    free(B);
}

void oracle_decode_xq(const int32_t *xqd, int32_t *xq, int eps) { /* svt_decode_xq (EbRestoration.c:634-646) */
    if (kSgrR[eps][0] == 0) {
        xq[0] = 0;
        xq[1] = (1 << 7) - xqd[1];
    } else if (kSgrR[eps][1] == 0) {
        xq[0] = xqd[0];
        xq[1] = 0;
    } else {
        xq[0] = xqd[0];
        xq[1] = (1 << 7) - xq[0] - xqd[1];
    }
}

/* apply_selfguided_restoration: dat readable at rows -3..h+2, cols -3..w+2 */
void oracle_sgr_apply(const uint16_t *dat, int stride, int w, int h, int eps, const int32_t *xqd, uint16_t *dst,
                      int dstride, int bd) {
    const int es = w + 6;
    int32_t  *d  = malloc(sizeof(int32_t) * (size_t)es * (h + 6));
    int32_t  *f0 = malloc(sizeof(int32_t) * (size_t)w * h), *f1 = malloc(sizeof(int32_t) * (size_t)w * h);
    for (int i = -3; i < h + 3; i++)
        for (int j = -3; j < w + 3; j++) d[(i + 3) * es + j + 3] = dat[(long)i * stride + j];
    oracle_sgr_filter(d + 3 * es + 3, es, w, h, eps, bd, f0, f1, w);
    int32_t xq[2];
    oracle_decode_xq(xqd, xq, eps);
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            const int32_t u = (int32_t)dat[(long)i * stride + j] << 4;
            int32_t       v = u << 7;
            if (kSgrR[eps][0] > 0) v += xq[0] * (f0[i * w + j] - u);
            if (kSgrR[eps][1] > 0) v += xq[1] * (f1[i * w + j] - u);
            const int16_t o = (int16_t)((v + (1 << 10)) >> 11);
            dst[(long)i * dstride + j] = (uint16_t)CLAMP_(o, 0, (1 << bd) - 1);
        }
    free(d);
    free(f0);
    free(f1);
}

/* ------------------------------------------------------------------------------------------- */
/* frame apply                                                                                  */
/* ------------------------------------------------------------------------------------------- */
static int plane_px(const OracleFrame *f, int p, int y, int x) {
    const long i = (long)y * f->stride[p] + x;
    return f->bit_depth > 8 ? ((const uint16_t *)f->plane[p])[i] : ((const uint8_t *)f->plane[p])[i];
}
static void set_px(OracleFrame *f, int p, int y, int x, int v) {
    const long i = (long)y * f->stride[p] + x;
    if (f->bit_depth > 8)
        ((uint16_t *)f->plane[p])[i] = (uint16_t)v;
    else
        ((uint8_t *)f->plane[p])[i] = (uint8_t)v;
}

int oracle_lr_units(int size, int extent) { return MAX_((extent + (size >> 1)) / size, 1); }

/* One plane of svt_av1_loop_restoration_filter_frame: out = restored cdef (units/types), boundary lines from
 * dlf rows around internal stripe edges. */
static void lr_plane(const OracleFrame *dlf, const OracleFrame *cdef, OracleFrame *out, int p, int unit_size,
                     const SvtGpuRestUnit *units) {
    const int ss = p > 0, W = p ? (cdef->width + 1) >> 1 : cdef->width, H = p ? (cdef->height + 1) >> 1 : cdef->height;
    const int bd = cdef->bit_depth;
    const int full = 64 >> ss, off = 8 >> ss, procw = 64 >> ss;
    const int hunits = oracle_lr_units(unit_size, W);
    const int ext    = unit_size * 3 / 2;
    int       r0, r1;
    oracle_wiener_round(bd, &r0, &r1);
    /* foreach_rest_unit_in_tile (EbRestoration.c:1257-1294) */
    for (int y0 = 0, ui = 0; y0 < H; ui++) {
        const int uh = (H - y0 < ext) ? H - y0 : unit_size;
        int       vs = MAX_(0, y0 - off), ve = y0 + uh;
        if (ve < H) ve -= off;
        for (int x0 = 0, uj = 0; x0 < W; uj++) {
            const int             uw = (W - x0 < ext) ? W - x0 : unit_size;
            const SvtGpuRestUnit *u  = &units[ui * hunits + uj];
            if (u->type == SVTGPU_RESTORE_NONE) {
                for (int y = vs; y < ve; y++)
                    for (int x = x0; x < x0 + uw; x++) set_px(out, p, y, x, plane_px(cdef, p, y, x));
                x0 += uw;
                continue;
            }
            /* svt_av1_loop_restoration_filter_unit: one processing stripe at a time */
            for (int i = 0; i < ve - vs;) {
                const int v_start   = vs + i;
                const int first     = v_start == 0;
                const int this_h    = full - (first ? off : 0);
                const int copy_abv  = !first, copy_blw = !(v_start + this_h >= H);
                const int tstripe   = (v_start + off) / full;
                const int h         = MIN_(full - (tstripe == 0 ? off : 0), ve - v_start);
                const int vw        = ((uw + 15) & ~15) + 8; /* virtual columns -3 .. round16(uw)+4 */
                const int vh        = h + 7;                  /* virtual rows -3 .. h+3 */
                uint16_t *virt      = malloc(sizeof(uint16_t) * (size_t)vw * vh);
                for (int r = -3; r < h + 4; r++) {
                    const OracleFrame *srcf = cdef;
                    int                sy   = CLAMP_(v_start + r, 0, H - 1);
                    if (r < 0 && copy_abv) { /* (L0, L0, L1): deblocked rows v_start-2, v_start-1 */
                        srcf = dlf;
                        sy   = v_start + (r == -1 ? -1 : -2);
                    } else if (r >= h && r < h + 3 && copy_blw) { /* (B0, B1, B1) */
                        srcf = dlf;
                        sy   = MIN_(v_start + h + (r == h ? 0 : 1), H - 1);
                    }
                    for (int c = -3; c < vw - 3; c++)
                        virt[(r + 3) * vw + c + 3] = (uint16_t)plane_px(srcf, p, sy, CLAMP_(x0 + c, 0, W - 1));
                }
                const uint16_t *v0  = virt + 3 * vw + 3;
                uint16_t       *res = malloc(sizeof(uint16_t) * (size_t)vw * h);
                for (int j = 0; j < uw; j += procw) {
                    if (u->type == SVTGPU_RESTORE_WIENER) {
                        const int w = MIN_(procw, (uw - j + 15) & ~15);
                        oracle_wiener_convolve(v0 + j, vw, res + j, vw, u->hfilter, u->vfilter, w, h, r0, r1, bd);
                    } else {
                        const int w = MIN_(procw, uw - j);
                        oracle_sgr_apply(v0 + j, vw, w, h, u->ep, u->xqd, res + j, vw, bd);
                    }
                }
                for (int y = 0; y < h; y++)
                    for (int x = 0; x < uw; x++) set_px(out, p, v_start + y, x0 + x, res[y * vw + x]);
                free(res);
                free(virt);
                i += h;
            }
            x0 += uw;
        }
        y0 += uh;
    }
}

int oracle_lr_apply_frame(const OracleFrame *dlf, const OracleFrame *cdef, OracleFrame *out, const int *frame_type,
                          const int *unit_size, const SvtGpuRestUnit *const *units) {
    for (int p = 0; p < 3; p++) {
        const int W = p ? (cdef->width + 1) >> 1 : cdef->width, H = p ? (cdef->height + 1) >> 1 : cdef->height;
        if (frame_type[p] == SVTGPU_RESTORE_NONE) {
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) set_px(out, p, y, x, plane_px(cdef, p, y, x));
            continue;
        }
        lr_plane(dlf, cdef, out, p, unit_size[p], units[p]);
    }
    return SVTGPU_OK;
}
