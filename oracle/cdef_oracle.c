/*
 * cdef_oracle.c — CPU restatement of SVT-AV1 v2.1.0's CDEF search / pick / apply.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity is pinned by tests/test_oracle_golden.py
 * against vectors generated from the reference's own C kernels (oracle/ref.mk).
 *
 * Citations are Source/Lib/<path>:<line> in the reference checkout.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MIN_(a, b) ((a) < (b) ? (a) : (b))
#define MAX_(a, b) ((a) > (b) ? (a) : (b))

static int msb32(uint32_t v) { /* get_msb (EbUtility.h): index of the highest set bit, v > 0 */
    int n = 0;
    while (v >>= 1) n++;
    return n;
}

/* ------------------------------------------------------------------------------------------- */
/* Direction search — Common/Codec/EbCdef.c:150-210                                             */
/* ------------------------------------------------------------------------------------------- */
uint8_t oracle_cdef_find_dir(const uint16_t *img, int32_t stride, int32_t *var, int32_t coeff_shift) {
    /* 840/n weights (EbCdef.c:163) */
    static const int32_t w840[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
    int32_t line[8][15];
    int32_t cost[8];
    memset(line, 0, sizeof(line));
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) {
            const int32_t v = (img[r * stride + c] >> coeff_shift) - 128;
            line[0][r + c] += v;
            line[1][r + c / 2] += v;
            line[2][r] += v;
            line[3][3 + r - c / 2] += v;
            line[4][7 + r - c] += v;
            line[5][3 - r / 2 + c] += v;
            line[6][c] += v;
            line[7][r / 2 + c] += v;
        }
    /* horizontal / vertical: 8 full lines (EbCdef.c:183-188) */
    int32_t h = 0, v = 0;
    for (int k = 0; k < 8; k++) {
        h += line[2][k] * line[2][k];
        v += line[6][k] * line[6][k];
    }
    cost[2] = h * w840[8];
    cost[6] = v * w840[8];
    /* diagonals: lines of length 1..8 (EbCdef.c:189-194) */
    cost[0] = line[0][7] * line[0][7] * w840[8];
    cost[4] = line[4][7] * line[4][7] * w840[8];
    for (int k = 0; k < 7; k++) {
        cost[0] += (line[0][k] * line[0][k] + line[0][14 - k] * line[0][14 - k]) * w840[k + 1];
        cost[4] += (line[4][k] * line[4][k] + line[4][14 - k] * line[4][14 - k]) * w840[k + 1];
    }
    /* odd directions: 5 full-length lines + 3 pairs of partial lines (EbCdef.c:195-203) */
    for (int d = 1; d < 8; d += 2) {
        int32_t full = 0;
        for (int k = 3; k < 8; k++) full += line[d][k] * line[d][k];
        cost[d] = full * w840[8];
        for (int k = 0; k < 3; k++)
            cost[d] += (line[d][k] * line[d][k] + line[d][10 - k] * line[d][10 - k]) * w840[2 * k + 2];
    }
    /* first strict maximum (EbCdef.c:204-209) */
    int32_t best = 0;
    uint8_t bd   = 0;
    for (int d = 0; d < 8; d++)
        if (cost[d] > best) {
            best = cost[d];
            bd   = (uint8_t)d;
        }
    *var = (best - cost[(bd + 4) & 7]) >> 10;
    return bd;
}

/* ------------------------------------------------------------------------------------------- */
/* Directional filter — Common/Codec/EbCdef.c:85-135, 249-300                                  */
/* ------------------------------------------------------------------------------------------- */
/* Cdef_Directions with the +-2 index padding of EbCdef.c:99-122, expressed as (dy, dx) pairs */
static const int8_t k_dir_dy_dx[12][2][2] = {
    {{1, 0}, {2, 0}},   {{1, 0}, {2, -1}}, /* padding = dirs 6, 7 */
    {{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, {{0, 1}, {0, 2}}, {{0, 1}, {1, 2}},
    {{1, 1}, {2, 2}},   {{1, 0}, {2, 1}},  {{1, 0}, {2, 0}}, {{1, 0}, {2, -1}},
    {{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, /* padding = dirs 0, 1 */
};
static int dir_offset(int dir, int k, int stride) { /* svt_aom_eb_cdef_directions[dir][k] */
    const int8_t *o = k_dir_dy_dx[dir + 2][k];
    return o[0] * stride + o[1];
}

static int32_t constrain_(int32_t diff, int32_t threshold, int32_t damping) { /* EbCdef.c:85-91 */
    if (!threshold)
        return 0;
    const int32_t shift = MAX_(0, damping - msb32((uint32_t)threshold));
    const int32_t mag   = MIN_(abs(diff), MAX_(0, threshold - (abs(diff) >> shift)));
    return diff < 0 ? -mag : mag;
}

static int32_t adjust_strength_(int32_t strength, int32_t var) { /* EbCdef.c:130-135 */
    const int32_t i = (var >> 6) ? MIN_(msb32((uint32_t)(var >> 6)), 12) : 0;
    return var ? (strength * (4 + i) + 8) >> 4 : 0;
}

void oracle_cdef_filter_block(uint8_t *dst8, uint16_t *dst16, int32_t dstride, const uint16_t *in,
                              int32_t pri_strength, int32_t sec_strength, int32_t dir, int32_t pri_damping,
                              int32_t sec_damping, int32_t bsize, int32_t coeff_shift, uint8_t subsampling_factor) {
    static const int32_t pri_taps[2][2] = {{4, 2}, {3, 3}}; /* EbCdef.c:249 */
    static const int32_t sec_taps[2][2] = {{2, 1}, {2, 1}}; /* EbCdef.c:250 */
    const int      s   = OR_CDEF_BSTRIDE;
    const int32_t *pt  = pri_taps[(pri_strength >> coeff_shift) & 1];
    const int32_t *st  = sec_taps[(pri_strength >> coeff_shift) & 1];
    const int      bh  = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_4X8) ? 8 : 4;
    const int      bw  = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_8X4) ? 8 : 4;
    for (int i = 0; i < bh; i += subsampling_factor) {
        for (int j = 0; j < bw; j++) {
            const uint16_t *p   = in + i * s + j;
            const int16_t   x   = (int16_t)p[0];
            int16_t         sum = 0; /* int16 accumulation as in EbCdef.c:263 */
            int32_t         hi  = x, lo = x;
            for (int k = 0; k < 2; k++) {
                const int op  = dir_offset(dir, k, s);
                const int os0 = dir_offset(dir + 2, k, s);
                const int os1 = dir_offset(dir - 2, k, s);
                const int16_t taps_p[2] = {(int16_t)p[op], (int16_t)p[-op]};
                const int16_t taps_s[4] = {(int16_t)p[os0], (int16_t)p[-os0], (int16_t)p[os1], (int16_t)p[-os1]};
                for (int t = 0; t < 2; t++) {
                    sum += (int16_t)(pt[k] * constrain_(taps_p[t] - x, pri_strength, pri_damping));
                    if (taps_p[t] != OR_CDEF_VERY_LARGE)
                        hi = MAX_(hi, taps_p[t]);
                    lo = MIN_(lo, taps_p[t]);
                }
                for (int t = 0; t < 4; t++) {
                    if (taps_s[t] != OR_CDEF_VERY_LARGE)
                        hi = MAX_(hi, taps_s[t]);
                    lo = MIN_(lo, taps_s[t]);
                    sum += (int16_t)(st[k] * constrain_(taps_s[t] - x, sec_strength, sec_damping));
                }
            }
            int32_t y = (int16_t)x + ((8 + sum - (sum < 0)) >> 4);
            y         = y < lo ? lo : (y > hi ? hi : y);
            if (dst8)
                dst8[i * dstride + j] = (uint8_t)y;
            else
                dst16[i * dstride + j] = (uint16_t)y;
        }
    }
}

/* ------------------------------------------------------------------------------------------- */
/* Distortion — Encoder/Codec/EbEncCdef.c:23-219                                                */
/* ------------------------------------------------------------------------------------------- */
/* SSIM-like luma term of dist_8xn_*_c (EbEncCdef.c:23-48).  `flt` is the packed filtered block
 * (stride 8), `org` the source at stride `ostride`.  Same operand order as the reference so the
 * double-precision evaluation matches bit for bit. */
static uint64_t luma_dist_8xn(const uint64_t sum_s, const uint64_t sum_d, const uint64_t sum_s2,
                              const uint64_t sum_d2, const uint64_t sum_sd, int32_t coeff_shift) {
    const uint64_t svar = sum_s2 - ((sum_s * sum_s + 32) >> 6);
    const uint64_t dvar = sum_d2 - ((sum_d * sum_d + 32) >> 6);
    return (uint64_t)floor(.5 + (sum_d2 + sum_s2 - 2 * sum_sd) * .5 * (svar + dvar + (400 << 2 * coeff_shift)) /
                                    (sqrt((20000 << 4 * coeff_shift) + svar * (double)dvar)));
}

#define DEFINE_CDEF_DIST(NAME, T)                                                                           \
    uint64_t NAME(const T *dst, int32_t dstride, const T *src, const SvtGpuCdefList *dlist, int32_t cdef_count, \
                  int32_t bsize, int32_t coeff_shift, int32_t pli, uint8_t ss) {                            \
        const int bh = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_4X8) ? 8 : 4;                   \
        const int bw = (bsize == SVTGPU_BLOCK_8X8 || bsize == SVTGPU_BLOCK_8X4) ? 8 : 4;                   \
        const int lbh = bh == 8 ? 3 : 2, lbw = bw == 8 ? 3 : 2;                                            \
        uint64_t  total = 0;                                                                               \
        for (int bi = 0; bi < cdef_count; bi++) {                                                          \
            const T *f = src + (bi << (lbh + lbw));                       /* packed filtered block */      \
            const T *o = dst + (dlist[bi].by << lbh) * dstride + (dlist[bi].bx << lbw); /* source */        \
            if (bsize == SVTGPU_BLOCK_8X8 && pli == 0) {                                                   \
                uint64_t s1 = 0, d1 = 0, s2 = 0, d2 = 0, sd = 0;                                           \
                for (int i = 0; i < 8; i += ss)                                                            \
                    for (int j = 0; j < 8; j++) {                                                          \
                        const uint64_t a = f[8 * i + j], b = o[i * dstride + j];                          \
                        s1 += a; d1 += b; s2 += a * a; d2 += b * b; sd += a * b;                          \
                    }                                                                                      \
                total += luma_dist_8xn(s1, d1, s2, d2, sd, coeff_shift);                                   \
            } else {                                                                                       \
                for (int i = 0; i < bh; i += ss)                                                           \
                    for (int j = 0; j < bw; j++) {                                                         \
                        const int32_t e = (int32_t)o[i * dstride + j] - (int32_t)f[bw * i + j];           \
                        total += (uint64_t)(e * e);                                                        \
                    }                                                                                      \
            }                                                                                              \
        }                                                                                                  \
        return total >> (2 * coeff_shift);                                                                 \
    }
DEFINE_CDEF_DIST(oracle_compute_cdef_dist_16bit, uint16_t)
DEFINE_CDEF_DIST(oracle_compute_cdef_dist_8bit, uint8_t)

/* ------------------------------------------------------------------------------------------- */
/* Strength-pair greedy — EbEncCdef.c:627-728                                                   */
/* ------------------------------------------------------------------------------------------- */
uint64_t oracle_search_one_dual(int *lev0, int *lev1, int nb_strengths, uint64_t **mse[2], int sb_count,
                                int start_gi, int end_gi) {
    const int n   = end_gi;
    uint64_t *tot = (uint64_t *)calloc((size_t)64 * 64, sizeof(uint64_t));
    for (int fb = 0; fb < sb_count; fb++) {
        uint64_t best = (uint64_t)1 << 63;
        for (int g = 0; g < nb_strengths; g++) {
            const uint64_t c = mse[0][fb][lev0[g]] + mse[1][fb][lev1[g]];
            if (c < best)
                best = c;
        }
        for (int j = start_gi; j < n; j++)
            for (int k = start_gi; k < n; k++) {
                const uint64_t c = mse[0][fb][j] + mse[1][fb][k];
                tot[j * 64 + k] += c < best ? c : best;
            }
    }
    uint64_t best_tot = (uint64_t)1 << 63;
    int      b0 = 0, b1 = 0;
    for (int j = start_gi; j < n; j++)
        for (int k = start_gi; k < n; k++)
            if (tot[j * 64 + k] < best_tot) { /* first minimum wins (EbEncCdef.c:670-679) */
                best_tot = tot[j * 64 + k];
                b0       = j;
                b1       = k;
            }
    lev0[nb_strengths] = b0;
    lev1[nb_strengths] = b1;
    free(tot);
    return best_tot;
}

static uint64_t joint_search_(int *lev0, int *lev1, int nb, uint64_t **mse[2], int sb_count, int start_gi,
                              int end_gi) { /* EbEncCdef.c:697-727 */
    uint64_t r = (uint64_t)1 << 63;
    for (int i = 0; i < nb; i++) r = oracle_search_one_dual(lev0, lev1, i, mse, sb_count, start_gi, end_gi);
    for (int i = 0; i < 4 * nb; i++) {
        for (int j = 0; j < nb - 1; j++) {
            lev0[j] = lev0[j + 1];
            lev1[j] = lev1[j + 1];
        }
        r = oracle_search_one_dual(lev0, lev1, nb - 1, mse, sb_count, start_gi, end_gi);
    }
    return r;
}

/* ------------------------------------------------------------------------------------------- */
/* Controls — Encoder/Codec/EncModeConfig.c:12, 860-1330                                        */
/* ------------------------------------------------------------------------------------------- */
int oracle_cdef_controls_for_level(int level, SvtGpuCdefControls *c) {
    static const uint8_t pf[16] = {0, 4, 8, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48, 52, 56, 60};
    /* first-pass primary indices per level, second-pass secondary set, uv flags, ss, bias */
    static const int8_t first_sets[11][17] = {
        /* n, idx... */
        {16, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, /* L1 */
        {12, 0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14},              /* L2 */
        {8, 0, 2, 4, 6, 8, 10, 12, 14},                            /* L3 */
        {5, 0, 4, 8, 12, 15},                                      /* L4 */
        {4, 0, 5, 10, 15},                                         /* L5 */
        {3, 0, 7, 15},                                             /* L6 */
        {3, 0, 7, 15},                                             /* L7 */
        {3, 0, 7, 15},                                             /* L8 */
        {2, 0, 15},                                                /* L9, L10, L12, L13, L16 (+ L11, L14) */
        {1, 0},                                                    /* L15, L17 */
    };
    memset(c, 0, sizeof(*c));
    int set, nsec, sec_uv_on, first_uv_on = 1;
    int sec_list[3] = {1, 2, 3};
    switch (level) {
    case 1: set = 0, nsec = 3, sec_uv_on = 1, c->subsampling_factor = 1; break;
    case 2: set = 1, nsec = 3, sec_uv_on = 0, c->subsampling_factor = 1; break;
    case 3: set = 2, nsec = 3, sec_uv_on = 1, c->subsampling_factor = 1; break;
    case 4: set = 3, nsec = 3, sec_uv_on = 0, c->subsampling_factor = 1; break;
    case 5: set = 4, nsec = 3, sec_uv_on = 1, c->subsampling_factor = 1; break;
    case 6: set = 5, nsec = 3, sec_uv_on = 0, c->subsampling_factor = 1; break;
    case 7: set = 6, nsec = 2, sec_uv_on = 1, c->subsampling_factor = 1; break;
    case 8:
        set = 7, nsec = 1, sec_uv_on = 0, c->subsampling_factor = 1;
        sec_list[0] = 2;
        break;
    case 9:
    case 10:
    case 12:
    case 13:
    case 16:
        set = 8, nsec = 1, sec_uv_on = 0, c->subsampling_factor = 4;
        sec_list[0] = 2;
        c->zero_fs_cost_bias = (level >= 12) ? 62 : 0;
        break;
    case 11: /* use_reference_cdef_fs levels: the controls of :1108-1267, no search at run time */
    case 14:
        set = 8, nsec = 1, sec_uv_on = 0, c->subsampling_factor = 4;
        sec_list[0] = 2;
        c->zero_fs_cost_bias     = level == 14 ? 62 : 0;
        c->use_reference_cdef_fs = 1;
        break;
    case 15:
    case 17:
        set = 9, nsec = 0, sec_uv_on = 0, c->subsampling_factor = 4;
        c->zero_fs_cost_bias     = 62;
        c->use_reference_cdef_fs = 1;
        break;
    default: return SVTGPU_ERR_UNSUPPORTED; /* 0 = off */
    }
    const int8_t *fs = first_sets[set];
    c->first_pass_fs_num          = (uint8_t)fs[0];
    c->default_second_pass_fs_num = (uint8_t)(fs[0] * nsec);
    int sf                        = 0;
    for (int i = 0; i < fs[0]; i++) {
        c->default_first_pass_fs[i]    = pf[fs[1 + i]];
        c->default_first_pass_fs_uv[i] = first_uv_on ? (int8_t)pf[fs[1 + i]] : -1;
        for (int j = 0; j < nsec; j++, sf++) {
            c->default_second_pass_fs[sf]    = (uint8_t)(pf[fs[1 + i]] + sec_list[j]);
            c->default_second_pass_fs_uv[sf] = sec_uv_on ? (int8_t)c->default_second_pass_fs[sf] : -1;
        }
    }
    return SVTGPU_OK;
}

/* ------------------------------------------------------------------------------------------- */
/* Frame geometry helpers                                                                        */
/* ------------------------------------------------------------------------------------------- */
typedef struct Geo {
    int mi_rows, mi_cols, nvfb, nhfb, b8_rows, b8_cols;
} Geo;
static Geo geo_of(int32_t w, int32_t h) {
    Geo g;
    g.mi_cols = ((w + 7) & ~7) >> 2; /* mi units of 4 px, frame aligned to 8 */
    g.mi_rows = ((h + 7) & ~7) >> 2;
    g.nhfb    = (g.mi_cols + 15) / 16;
    g.nvfb    = (g.mi_rows + 15) / 16;
    g.b8_cols = g.mi_cols / 2;
    g.b8_rows = g.mi_rows / 2;
    return g;
}

/* svt_sb_compute_cdef_list (EbEncCdef.c:238-282) over a per-8x8 mask: the listed 8x8 blocks of the area of
 * nvb x nhb mi units at filter block (fbr, fbc) (16 x 16 for a 64x64 block, up to 32 for 128-wide SB128 blocks) */
static int fb_block_list(const Geo *g, const uint8_t *mask, int fbr, int fbc, int nvb, int nhb, SvtGpuCdefList *dl) {
    int n = 0;
    for (int r = 0; r < nvb; r += 2)
        for (int c = 0; c < nhb; c += 2) {
            const int br = 8 * fbr + r / 2, bc = 8 * fbc + c / 2;
            if (!mask || mask[br * g->b8_cols + bc]) {
                dl[n].by = (uint8_t)(r >> 1);
                dl[n].bx = (uint8_t)(c >> 1);
                n++;
            }
        }
    return n;
}

static void stage_rect(uint16_t *dst, int dstride, const OracleFrame *f, int pli, int row, int col, int rows,
                       int cols) { /* svt_aom_copy_sb8_16 (EbCdef.c:314-333) */
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) {
            const long idx = (long)(row + r) * f->stride[pli] + (col + c);
            dst[r * dstride + c] = f->bit_depth > 8 ? ((const uint16_t *)f->plane[pli])[idx]
                                                    : ((const uint8_t *)f->plane[pli])[idx];
        }
}

/* cdef_find_dir over the list (EbCdef.c:218-247) + the per-FB driver svt_cdef_filter_fb
 * (EbCdef.c:339-430) for 4:2:0 and the packed (dstride == 0) search output */
static void filter_fb_packed(void *dst, int is16, const uint16_t *in, int pli, const SvtGpuCdefList *dl, int n,
                             uint8_t dir[16][16], int32_t var[16][16], int *dirinit, int level, int sec, int damping,
                             int cs, int ss) {
    const int xdec = pli ? 1 : 0, ydec = xdec;
    int       pri  = level << cs;
    sec <<= cs;
    const int pdamp = damping + cs - (pli != 0), sdamp = pdamp;
    const int bsize = ydec ? SVTGPU_BLOCK_4X4 : SVTGPU_BLOCK_8X8;
    const int lbx = 3 - xdec, lby = 3 - ydec;
    if (pri == 0 && sec == 0) { /* plain copy path (EbCdef.c:358-383) */
        for (int bi = 0; bi < n; bi++) {
            const uint16_t *s = in + (dl[bi].by << lby) * OR_CDEF_BSTRIDE + (dl[bi].bx << lbx);
            for (int iy = 0; iy < (1 << lby); iy += ss)
                for (int ix = 0; ix < (1 << lbx); ix++) {
                    const int o = (bi << (lbx + lby)) + (iy << lbx) + ix;
                    if (is16)
                        ((uint16_t *)dst)[o] = s[iy * OR_CDEF_BSTRIDE + ix];
                    else
                        ((uint8_t *)dst)[o] = (uint8_t)s[iy * OR_CDEF_BSTRIDE + ix];
                }
        }
        return;
    }
    if (pli == 0 && !*dirinit) {
        for (int bi = 0; bi < n; bi++) {
            const int by = dl[bi].by, bx = dl[bi].bx;
            dir[by][bx] = oracle_cdef_find_dir(in + 8 * by * OR_CDEF_BSTRIDE + 8 * bx, OR_CDEF_BSTRIDE, &var[by][bx], cs);
        }
        *dirinit = 1;
    }
    for (int bi = 0; bi < n; bi++) {
        const int by = dl[bi].by, bx = dl[bi].bx;
        const int t  = pli ? pri : adjust_strength_(pri, var[by][bx]);
        const int d  = pri ? dir[by][bx] : 0;
        const uint16_t *src = in + (by << lby) * OR_CDEF_BSTRIDE + (bx << lbx);
        const int o = bi << (lbx + lby);
        if (is16)
            oracle_cdef_filter_block(NULL, (uint16_t *)dst + o, 1 << lbx, src, t, sec, d, pdamp, sdamp, bsize, cs, (uint8_t)ss);
        else
            oracle_cdef_filter_block((uint8_t *)dst + o, NULL, 1 << lbx, src, t, sec, d, pdamp, sdamp, bsize, cs, (uint8_t)ss);
    }
}

/* ------------------------------------------------------------------------------------------- */
/* Search — Encoder/Codec/EbCdefProcess.c:114-357 (all segments).  fb_bsize (NULL = SB64) is the BlockSize of */
/* the mode info at each filter block's top-left: a 128x128 / 128x64 / 64x128 block is searched as one area   */
/* (:188-205) whose list and distortion land in its top-left filter block; the other halves are left out of   */
/* the pick (skip = 1 here).  dir / var are stored per 64x64 filter block, 8x8 blocks row-major.               */
/* ------------------------------------------------------------------------------------------- */
int oracle_cdef_search_frame_sb(const OracleFrame *recon, const OracleFrame *src, const uint8_t *block_mask,
                                const uint8_t *fb_bsize, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                                uint64_t *mse, uint8_t *skip, uint8_t *dir_out, int32_t *var_out) {
    const Geo g      = geo_of(recon->width, recon->height);
    const int nfb    = g.nvfb * g.nhfb;
    const int cs     = recon->bit_depth > 8 ? recon->bit_depth - 8 : 0;
    const int is16   = recon->bit_depth > 8;
    const int damp   = 3 + (base_q_idx >> 6);
    /* use_reference_cdef_fs: no strength search (EbCdefProcess.c:400); only the directions the apply needs */
    const int ref_fs = ctrls->use_reference_cdef_fs;
    const int nfirst = ref_fs ? 0 : ctrls->first_pass_fs_num, nsec = ref_fs ? 0 : ctrls->default_second_pass_fs_num;
    uint16_t *inbuf  = (uint16_t *)malloc(sizeof(uint16_t) * OR_CDEF_INBUF_SIZE);
    uint16_t *tmp    = (uint16_t *)malloc(sizeof(uint16_t) * 128 * 128);
    SvtGpuCdefList dl[256];
    uint16_t      *in = inbuf + OR_CDEF_VBORDER * OR_CDEF_BSTRIDE + OR_CDEF_HBORDER;
    for (int fbr = 0; fbr < g.nvfb; fbr++)
        for (int fbc = 0; fbc < g.nhfb; fbc++) {
            const int fb = fbr * g.nhfb + fbc;
            const int bs = fb_bsize ? fb_bsize[fb] : 0; /* 13 64X128, 14 128X64, 15 128X128 */
            uint64_t *m0 = mse + (size_t)fb * 64, *m1 = mse + ((size_t)nfb + fb) * 64;
            if (((fbc & 1) && (bs == 15 || bs == 14)) || ((fbr & 1) && (bs == 15 || bs == 13))) {
                skip[fb] = 1; /* a half of a 128-wide area: searched with its top-left block (:193-196) */
                memset(m0, 0, 64 * sizeof(uint64_t));
                memset(m1, 0, 64 * sizeof(uint64_t));
                continue;
            }
            const int hb_step = (bs == 15 || bs == 14) ? 2 : 1, vb_step = (bs == 15 || bs == 13) ? 2 : 1;
            const int nhb = MIN_(16 * hb_step, g.mi_cols - 16 * fbc), nvb = MIN_(16 * vb_step, g.mi_rows - 16 * fbr);
            uint8_t   dir[16][16];
            int32_t   var[16][16];
            memset(dir, 0, sizeof(dir));
            memset(var, 0, sizeof(var));
            int       dirinit = 0;
            const int n = fb_block_list(&g, block_mask, fbr, fbc, nvb, nhb, dl);
            skip[fb] = n == 0;
            if (n == 0) {
                memset(m0, 0, 64 * sizeof(uint64_t));
                memset(m1, 0, 64 * sizeof(uint64_t));
                for (int by = 0; by < nvb / 2; by++) /* every 8x8 block of the area: not listed */
                    for (int bx = 0; bx < nhb / 2; bx++) {
                        const int f = (fbr + by / 8) * g.nhfb + fbc + bx / 8, k = (by % 8) * 8 + bx % 8;
                        dir_out[(size_t)f * 64 + k] = 0;
                        var_out[(size_t)f * 64 + k] = 0;
                    }
                continue;
            }
            for (int pli = 0; pli < 3; pli++) {
                const int sub = pli ? 1 : 0;
                if (pli < 2)
                    for (int i = 0; i < OR_CDEF_INBUF_SIZE; i++) inbuf[i] = OR_CDEF_VERY_LARGE;
                const int yoff  = OR_CDEF_VBORDER * (fbr != 0);
                const int xoff  = OR_CDEF_HBORDER * (fbc != 0);
                const int ysize = (nvb << (2 - sub)) + OR_CDEF_VBORDER * (fbr + vb_step < g.nvfb) + yoff;
                const int xsize = (nhb << (2 - sub)) + OR_CDEF_HBORDER * (fbc + hb_step < g.nhfb) + xoff;
                stage_rect(in - yoff * OR_CDEF_BSTRIDE - xoff, OR_CDEF_BSTRIDE, recon, pli, (16 * fbr << (2 - sub)) - yoff,
                           (16 * fbc << (2 - sub)) - xoff, ysize, xsize);
                int ss = ctrls->subsampling_factor;
                ss     = pli ? 1 : MIN_(ss, 4); /* caps of EbCdefProcess.c:254-259 (4:2:0) */
                const long soff = (long)(16 * fbr << (2 - sub)) * src->stride[pli] + (16 * fbc << (2 - sub));
                if (ref_fs && pli == 0) /* a throw-away filter pass (any primary strength) finds the block directions */
                    filter_fb_packed(tmp, is16, in, pli, dl, n, dir, var, &dirinit, 1, 0, damp, cs, ss);
                for (int gi = 0; gi < nfirst + nsec; gi++) {
                    const int first = gi < nfirst;
                    const int code  = first ? ctrls->default_first_pass_fs[gi] : ctrls->default_second_pass_fs[gi - nfirst];
                    const int uvon  = first ? ctrls->default_first_pass_fs_uv[gi] != -1
                                            : ctrls->default_second_pass_fs_uv[gi - nfirst] != -1;
                    if (pli && !uvon) {
                        m1[gi] = 1040400ull * 64; /* default_mse_uv * 64 (EbCdefProcess.c:86, 259) */
                        continue;
                    }
                    const int pri = code / 4, sec = code % 4;
                    filter_fb_packed(tmp, is16, in, pli, dl, n, dir, var, &dirinit, pri, sec + (sec == 3), damp, cs, ss);
                    uint64_t d;
                    const int bsz = pli ? SVTGPU_BLOCK_4X4 : SVTGPU_BLOCK_8X8;
                    if (is16)
                        d = oracle_compute_cdef_dist_16bit((const uint16_t *)src->plane[pli] + soff, src->stride[pli], tmp, dl,
                                                           n, bsz, cs, pli, (uint8_t)ss);
                    else
                        d = oracle_compute_cdef_dist_8bit((const uint8_t *)src->plane[pli] + soff, src->stride[pli],
                                                          (const uint8_t *)tmp, dl, n, bsz, cs, pli, (uint8_t)ss);
                    if (pli == 0)
                        m0[gi] = d * ss;
                    else if (pli == 1)
                        m1[gi] = d * ss;
                    else
                        m1[gi] += d * ss;
                }
                if (pli == 0 && nfirst + nsec == 0)
                    memset(m0, 0, 64 * sizeof(uint64_t));
            }
            if (nfirst + nsec < 64) {
                memset(m0 + nfirst + nsec, 0, (size_t)(64 - nfirst - nsec) * sizeof(uint64_t));
                memset(m1 + nfirst + nsec, 0, (size_t)(64 - nfirst - nsec) * sizeof(uint64_t));
            }
            for (int by = 0; by < nvb / 2; by++) /* the area's 8x8 blocks into their own filter blocks */
                for (int bx = 0; bx < nhb / 2; bx++) {
                    const int f = (fbr + by / 8) * g.nhfb + fbc + bx / 8, k = (by % 8) * 8 + bx % 8;
                    dir_out[(size_t)f * 64 + k] = dir[by][bx];
                    var_out[(size_t)f * 64 + k] = var[by][bx];
                }
        }
    free(inbuf);
    free(tmp);
    return SVTGPU_OK;
}

int oracle_cdef_search_frame(const OracleFrame *recon, const OracleFrame *src, const uint8_t *block_mask,
                             const SvtGpuCdefControls *ctrls, int32_t base_q_idx, uint64_t *mse, uint8_t *skip,
                             uint8_t *dir_out, int32_t *var_out) {
    return oracle_cdef_search_frame_sb(recon, src, block_mask, NULL, ctrls, base_q_idx, mse, skip, dir_out, var_out);
}

/* ------------------------------------------------------------------------------------------- */
/* Pick — finish_cdef_search (EbEncCdef.c:728-926), SB64, use_reference_cdef_fs == 0            */
/* ------------------------------------------------------------------------------------------- */
int oracle_cdef_pick(int32_t width, int32_t height, const uint64_t *mse_in, const uint8_t *skip,
                     const SvtGpuCdefControls *ctrls, int32_t base_q_idx, uint64_t lambda, SvtGpuCdefParams *params,
                     int8_t *fb_strength) {
    const Geo g   = geo_of(width, height);
    const int nfb = g.nvfb * g.nhfb;
    const int end = ctrls->first_pass_fs_num + ctrls->default_second_pass_fs_num;
    if (ctrls->use_reference_cdef_fs) { /* EbEncCdef.c:744-789 */
        memset(params, 0, sizeof(*params));
        memset(fb_strength, 0, (size_t)nfb);
        params->cdef_damping        = (uint8_t)(3 + (base_q_idx >> 6));
        params->cdef_y_strength[0]  = (uint8_t)ctrls->pred_y_f;
        params->cdef_uv_strength[0] = (uint8_t)ctrls->pred_uv_f;
        return SVTGPU_OK;
    }
    uint64_t *mse = (uint64_t *)malloc(sizeof(uint64_t) * 2 * 64 * (size_t)nfb);
    memcpy(mse, mse_in, sizeof(uint64_t) * 2 * 64 * (size_t)nfb);
    uint64_t **rows[2];
    rows[0]       = (uint64_t **)malloc(sizeof(uint64_t *) * (size_t)(nfb + 1));
    rows[1]       = (uint64_t **)malloc(sizeof(uint64_t *) * (size_t)(nfb + 1));
    int *fb_of    = (int *)malloc(sizeof(int) * (size_t)(nfb + 1));
    int  sb_count = 0;
    for (int fb = 0; fb < nfb; fb++) {
        fb_strength[fb] = 0;
        if (skip[fb])
            continue;
        rows[0][sb_count] = mse + (size_t)fb * 64;
        rows[1][sb_count] = mse + ((size_t)nfb + fb) * 64;
        fb_of[sb_count++] = fb;
    }
    if (ctrls->zero_fs_cost_bias) /* EbEncCdef.c:845-851 */
        for (int i = 0; i < sb_count; i++) {
            rows[0][i][0] = (ctrls->zero_fs_cost_bias * rows[0][i][0]) >> 6;
            rows[1][i][0] = (ctrls->zero_fs_cost_bias * rows[1][i][0]) >> 6;
        }
    memset(params, 0, sizeof(*params));
    uint64_t best_cost = (uint64_t)1 << 63;
    int      nbits     = 0;
    for (int i = 0; i <= 3; i++) {
        int            lev0[SVTGPU_CDEF_MAX_STRENGTHS] = {0}, lev1[SVTGPU_CDEF_MAX_STRENGTHS] = {0};
        const int      nb   = 1 << i;
        const uint64_t tot  = joint_search_(lev0, lev1, nb, rows, sb_count, 0, end);
        const int      bits = sb_count * i + nb * 6 * 2;                 /* CDEF_STRENGTH_BITS = 6 */
        const int64_t  rate = (int64_t)bits << 9;                          /* av1_cost_literal */
        const uint64_t cost = (uint64_t)((((rate * (int64_t)lambda) + 256) >> 9) + ((int64_t)(tot * 16) << 7)); /* RDCOST */
        if (cost < best_cost) {
            best_cost = cost;
            nbits     = i;
            for (int j = 0; j < nb; j++) {
                params->cdef_y_strength[j]  = (uint8_t)lev0[j];
                params->cdef_uv_strength[j] = (uint8_t)lev1[j];
            }
        }
    }
    const int nb      = 1 << nbits;
    params->cdef_bits = (uint8_t)nbits;
    for (int i = 0; i < sb_count; i++) {
        uint64_t best = (uint64_t)1 << 63;
        int      bg   = 0;
        for (int gi = 0; gi < nb; gi++) {
            const uint64_t c = rows[0][i][params->cdef_y_strength[gi]] + rows[1][i][params->cdef_uv_strength[gi]];
            if (c < best) {
                best = c;
                bg   = gi;
            }
        }
        fb_strength[fb_of[i]] = (int8_t)bg;
    }
    /* gi -> strength code (filter_map, EbEncCdef.c:911-919) */
    for (int i = 0; i < nb; i++) {
        const int y = params->cdef_y_strength[i], uv = params->cdef_uv_strength[i];
        const int nf = ctrls->first_pass_fs_num;
        params->cdef_y_strength[i]  = y < nf ? ctrls->default_first_pass_fs[y] : ctrls->default_second_pass_fs[y - nf];
        params->cdef_uv_strength[i] = uv < nf ? ctrls->default_first_pass_fs[uv] : ctrls->default_second_pass_fs[uv - nf];
    }
    params->cdef_damping = (uint8_t)(3 + (base_q_idx >> 6));
    free(mse);
    free(rows[0]);
    free(rows[1]);
    free(fb_of);
    return SVTGPU_OK;
}

/* ------------------------------------------------------------------------------------------- */
/* Apply — svt_av1_cdef_frame (EbEncCdef.c:284-610), SB64.  Written out-of-place: every         */
/* neighbour the reference reads is unfiltered (its linebuf/colbuf are saved before filtering,   */
/* :470-547), so filtering each FB from the unfiltered input is the same computation.            */
/* ------------------------------------------------------------------------------------------- */
int oracle_cdef_apply_frame(const OracleFrame *recon, OracleFrame *out, const uint8_t *block_mask, const uint8_t *dir_in,
                            const int32_t *var_in, const SvtGpuCdefParams *params, const int8_t *fb_strength) {
    const Geo g    = geo_of(recon->width, recon->height);
    const int cs   = recon->bit_depth > 8 ? recon->bit_depth - 8 : 0;
    const int is16 = recon->bit_depth > 8;
    uint16_t *inbuf = (uint16_t *)malloc(sizeof(uint16_t) * OR_CDEF_INBUF_SIZE);
    uint16_t *in    = inbuf + OR_CDEF_VBORDER * OR_CDEF_BSTRIDE + OR_CDEF_HBORDER;
    SvtGpuCdefList dl[64];
    /* start from a copy of the input (unfiltered blocks / FBs pass through) */
    for (int pli = 0; pli < 3; pli++) {
        const int pw = pli ? recon->width / 2 : recon->width, ph = pli ? recon->height / 2 : recon->height;
        for (int r = 0; r < ph; r++) {
            if (is16)
                memcpy((uint16_t *)out->plane[pli] + (long)r * out->stride[pli],
                       (const uint16_t *)recon->plane[pli] + (long)r * recon->stride[pli], 2 * (size_t)pw);
            else
                memcpy((uint8_t *)out->plane[pli] + (long)r * out->stride[pli],
                       (const uint8_t *)recon->plane[pli] + (long)r * recon->stride[pli], (size_t)pw);
        }
    }
    for (int fbr = 0; fbr < g.nvfb; fbr++)
        for (int fbc = 0; fbc < g.nhfb; fbc++) {
            const int fb = fbr * g.nhfb + fbc;
            const int si = fb_strength[fb];
            int       level = params->cdef_y_strength[si] / 4, sec = params->cdef_y_strength[si] % 4;
            int       uvl = params->cdef_uv_strength[si] / 4, uvs = params->cdef_uv_strength[si] % 4;
            sec += sec == 3;
            uvs += uvs == 3;
            if (level == 0 && sec == 0 && uvl == 0 && uvs == 0)
                continue;
            const int nhb = MIN_(16, g.mi_cols - 16 * fbc), nvb = MIN_(16, g.mi_rows - 16 * fbr);
            const int n = fb_block_list(&g, block_mask, fbr, fbc, nvb, nhb, dl);
            if (n == 0)
                continue;
            uint8_t dir[8][8];
            int32_t var[8][8];
            memcpy(dir, dir_in + (size_t)fb * 64, 64);
            memcpy(var, var_in + (size_t)fb * 64, 64 * sizeof(int32_t));
            for (int pli = 0; pli < 3; pli++) {
                const int sub = pli ? 1 : 0;
                const int lv = pli ? uvl : level, sv = pli ? uvs : sec;
                if (!(lv || sv))
                    continue;
                const int hsize = nhb << (2 - sub), vsize = nvb << (2 - sub);
                const int r0 = 16 * fbr << (2 - sub), c0 = 16 * fbc << (2 - sub);
                /* unfiltered neighbourhood with 0x7F7F outside the frame (EbEncCdef.c:470-568) */
                for (int r = -OR_CDEF_VBORDER; r < vsize + OR_CDEF_VBORDER; r++)
                    for (int c = -OR_CDEF_HBORDER; c < hsize + OR_CDEF_HBORDER; c++) {
                        const int fr = r0 + r, fc = c0 + c;
                        const int ph = pli ? recon->height / 2 : recon->height;
                        const int pw = pli ? recon->width / 2 : recon->width;
                        uint16_t  v  = OR_CDEF_VERY_LARGE;
                        if (fr >= 0 && fc >= 0 && fr < ph && fc < pw) {
                            const long idx = (long)fr * recon->stride[pli] + fc;
                            v = is16 ? ((const uint16_t *)recon->plane[pli])[idx] : ((const uint8_t *)recon->plane[pli])[idx];
                        }
                        in[r * OR_CDEF_BSTRIDE + c] = v;
                    }
                const int pdamp = params->cdef_damping + cs - (pli != 0);
                const int pri = lv << cs, sst = sv << cs;
                const int lb = 3 - sub;
                for (int bi = 0; bi < n; bi++) {
                    const int by = dl[bi].by, bx = dl[bi].bx;
                    const int t  = pli ? pri : adjust_strength_(pri, var[by][bx]);
                    const long o = (long)(r0 + (by << lb)) * out->stride[pli] + c0 + (bx << lb);
                    const uint16_t *s = in + (by << lb) * OR_CDEF_BSTRIDE + (bx << lb);
                    const int bs = pli ? SVTGPU_BLOCK_4X4 : SVTGPU_BLOCK_8X8;
                    if (is16)
                        oracle_cdef_filter_block(NULL, (uint16_t *)out->plane[pli] + o, out->stride[pli], s, t, sst,
                                                 pri ? dir[by][bx] : 0, pdamp, pdamp, bs, cs, 1);
                    else
                        oracle_cdef_filter_block((uint8_t *)out->plane[pli] + o, NULL, out->stride[pli], s, t, sst,
                                                 pri ? dir[by][bx] : 0, pdamp, pdamp, bs, cs, 1);
                }
            }
        }
    free(inbuf);
    return SVTGPU_OK;
}
