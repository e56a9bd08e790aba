/*
 * me_oracle.c — CPU restatement of the open-loop ME SAD path (TEST INFRASTRUCTURE: imported only by tests/, smoke()
 * and bench.py's cpu_baseline leg; never shipped or measured).  Pinned by tests/golden/me_sad.bin, written by
 * oracle/ref_harness/gen_golden_me.c from the reference's own C.
 *
 *   oracle_me_search   open_loop_me_fullpel_search_sblock (EbMotionEstimation.c:782-818) per 64x64 block and
 *                      reference, after the best SADs are reset to MAX_SAD_VALUE (:1363-1364): per search row, groups
 *                      of 8 positions through the eight-point SADs (svt_ext_all_sad_calculation_8x8_16x16_c :336-368 +
 *                      svt_ext_eight_sad_calculation_32x32_64x64_c :370-428), the rest one position at a time
 *                      (svt_ext_sad_calculation_8x8_16x16_c :99-170 + svt_ext_sad_calculation_32x32_64x64_c :172-210).
 *                      The reference window is cut from the frame with edge replication (the padded reference).
 *   oracle_sad_loop    svt_sad_loop_kernel_c (EbComputeSAD_C.c:58-99).
 *   oracle_pme_sad_loop svt_pme_sad_loop_kernel_c (EbProductCodingLoop.c:1801-1852): the MD full-pel search, SAD plus
 *                      the MV rate of svt_aom_fp_mv_err_cost for each of the six MV_COST_TYPEs.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ME_MAX_SAD (128 * 128 * 255) /* MAX_SAD_VALUE, EbMotionEstimation.h:94 */

static uint32_t sad_rect(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
    uint32_t s = 0;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) s += (uint32_t)abs((int)a[y * as + x] - (int)b[y * bs + x]);
    return s;
}

/* 8x8 SAD (sub-sampled: rows 0, 2, 4, 6 of the 8x4-with-doubled-stride kernel, doubled) */
static uint32_t sad8(const uint8_t *s, int ss, const uint8_t *r, int rs, int sub) {
    return sub ? sad_rect(s, 2 * ss, r, 2 * rs, 8, 4) << 1 : sad_rect(s, ss, r, rs, 8, 8);
}

static uint32_t mv_add_x(uint32_t mv, int dx) {
    const int16_t x = (int16_t)(mv & 0xFFFF), y = (int16_t)(mv >> 16);
    return ((uint32_t)(uint16_t)y << 16) | (uint16_t)(int16_t)(x + dx);
}

/* one 64x64 block at one reference window: best[85] / mv[85] updated in the reference's scan order */
static void search_block(const uint8_t *src, int ss, const uint8_t *win, int ws, int ox, int oy, int saw, int sah,
                         int sub, uint32_t *best, uint32_t *bmv) {
    static const int zoff[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
    for (int k = 0; k < 85; k++) best[k] = ME_MAX_SAD, bmv[k] = 0;
    const int w8 = saw - (saw & 7);
    for (int y = 0; y < sah; y++) {
        for (int x = 0; x < saw; x += (x < w8 ? 8 : 1)) {
            const int      npos = x < w8 ? 8 : 1;
            const uint32_t mv   = ((uint32_t)(uint16_t)(int16_t)(oy + y) << 16) | (uint16_t)(int16_t)(ox + x);
            uint32_t       s16[16][8];
            for (int by = 0; by < 4; by++)
                for (int bx = 0; bx < 4; bx++) {
                    const int      q  = zoff[4 * by + bx];
                    const uint8_t *s  = src + 16 * by * ss + 16 * bx;
                    const uint8_t *r0 = win + (size_t)(y + 16 * by) * ws + x + 16 * bx;
                    for (int p = 0; p < npos; p++) {
                        const uint32_t m = npos == 8 ? mv_add_x(mv, p) : mv;
                        uint32_t       t = 0;
                        for (int k = 0; k < 4; k++) {
                            const int      o8 = 8 * (k >> 1) * ss + 8 * (k & 1), r8 = 8 * (k >> 1) * ws + 8 * (k & 1);
                            const uint32_t v  = sad8(s + o8, ss, r0 + p + r8, ws, sub);
                            if (v < best[4 * q + k]) best[4 * q + k] = v, bmv[4 * q + k] = m;
                            t += v;
                        }
                        if (t < best[64 + q]) best[64 + q] = t, bmv[64 + q] = m;
                        s16[q][p] = t;
                    }
                }
            for (int p = 0; p < npos; p++) {
                const uint32_t m   = npos == 8 ? mv_add_x(mv, p) : mv;
                uint32_t       s64 = 0;
                for (int k = 0; k < 4; k++) {
                    const uint32_t v = s16[4 * k][p] + s16[4 * k + 1][p] + s16[4 * k + 2][p] + s16[4 * k + 3][p];
                    if (v < best[80 + k]) best[80 + k] = v, bmv[80 + k] = m;
                    s64 += v;
                }
                if (s64 < best[84]) best[84] = s64, bmv[84] = m;
            }
        }
    }
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* src, refs: 8-bit luma planes W x H (stride = W); origin [nsb][nref][2]; out [nsb][nref][85] */
/* blocks [sb_begin, sb_end) only (outputs indexed from sb_begin) */
int oracle_me_search(const uint8_t *src, const uint8_t *const *refs, int nref, int W, int H, const int16_t *origin,
                     int saw, int sah, int sub, int sb_begin, int sb_end, uint32_t *best_sad, uint32_t *best_mv) {
    const int nsbx = (W + 63) / 64, ws = 64 + saw + 8, wh = 64 + sah;
    uint8_t  *win = malloc((size_t)ws * wh), sblk[64 * 64];
    if (!win) return -1;
    for (int sb = sb_begin; sb < sb_end; sb++) {
        const int sx0 = 64 * (sb % nsbx), sy0 = 64 * (sb / nsbx);
        for (int y = 0; y < 64; y++)
            for (int x = 0; x < 64; x++)
                sblk[y * 64 + x] = src[(size_t)clampi(sy0 + y, 0, H - 1) * W + clampi(sx0 + x, 0, W - 1)];
        for (int r = 0; r < nref; r++) {
            const size_t t  = (size_t)sb * nref + r;
            const int    ox = origin[2 * t], oy = origin[2 * t + 1];
            for (int y = 0; y < wh; y++)
                for (int x = 0; x < ws; x++)
                    win[(size_t)y * ws + x] =
                        refs[r][(size_t)clampi(sy0 + oy + y, 0, H - 1) * W + clampi(sx0 + ox + x, 0, W - 1)];
            const size_t o = ((size_t)(sb - sb_begin) * nref + r) * 85;
            search_block(sblk, 64, win, ws, ox, oy, saw, sah, sub, best_sad + o, best_mv + o);
        }
    }
    free(win);
    return 0;
}

/* svt_sad_loop_kernel_c: returns best sad (0xffffff when none is below it) and the centre */
void oracle_sad_loop(const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs, uint32_t bh, uint32_t bw,
                     uint64_t *best_sad, int16_t *xc, int16_t *yc, uint32_t src_stride_raw, uint8_t skip_search_line,
                     int16_t saw, int16_t sah) {
    *best_sad = 0xffffff;
    for (int y = 0; y < sah; y++) {
        if (bw == 16 && bh <= 16 && skip_search_line && (y & 1) == 0) continue;
        for (int x = 0; x < saw; x++) {
            const uint32_t s = sad_rect(src, (int)ss, ref + (size_t)y * src_stride_raw + x, (int)rs, (int)bw, (int)bh);
            if (s < *best_sad) *best_sad = s, *xc = (int16_t)x, *yc = (int16_t)y;
        }
    }
}

/* svt_pme_sad_loop_kernel_c (EbProductCodingLoop.c:1801-1852) with svt_aom_fp_mv_err_cost (mcomp.c:43-68, 771):
 * p = the reference's MV_COST_PARAMS (mcomp.h:37-48) read through its layout */
typedef struct {
    const int16_t *ref_mv; /* MV {row, col} */
    int16_t        full_ref_mv[2];
    uint8_t        mv_cost_type;
    const int     *mvjcost;
    const int     *mvcost[2];
    int            error_per_bit, early_exit_th, sad_per_bit;
} OracleMvCost;

static int mv_err_cost(int row, int col, const OracleMvCost *p) {
    const int dr = row - p->ref_mv[0], dc = col - p->ref_mv[1], ar = abs(dr), ac = abs(dc);
    switch (p->mv_cost_type) {
    case 0: {
        const int j = dr == 0 ? (dc == 0 ? 0 : 1) : (dc == 0 ? 2 : 3);
        const int r = dr < -(1 << 14) ? -(1 << 14) : dr > (1 << 14) ? (1 << 14) : dr;
        const int c = dc < -(1 << 14) ? -(1 << 14) : dc > (1 << 14) ? (1 << 14) : dc;
        const int64_t bits = (int64_t)p->mvjcost[j] + p->mvcost[0][r] + p->mvcost[1][c];
        return (int)((bits * p->error_per_bit + (1 << 13)) >> 14);
    }
    case 1: return (2 * (ar + ac)) >> 3;
    case 2: return 0;
    case 3: return (ar + ac) >> 3;
    case 4: return (int)(((int64_t)((ar + ac) << 8) * p->error_per_bit + (1 << 13)) >> 14);
    default: return 0;
    }
}

void oracle_pme_sad_loop(const void *params, const uint8_t *src, uint32_t ss, const uint8_t *ref, uint32_t rs,
                         uint32_t bh, uint32_t bw, uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                         int16_t sx, int16_t sy, int16_t saw, int16_t sah, int16_t step, int16_t mvx, int16_t mvy) {
    const OracleMvCost *p = (const OracleMvCost *)params;
    int col_num = 0, step_x = 1;
    for (int y = 0; y < sah; y += step) {
        for (int x = 0; x < saw; x += step_x) {
            if (saw - x < 8 && col_num == 0) continue;
            if (col_num == 7) col_num = 0, step_x = step;
            else col_num++, step_x = 1;
            const uint32_t cost0 = sad_rect(src, (int)ss, ref + (size_t)y * rs + x, (int)rs, (int)bw, (int)bh);
            const int16_t  col   = (int16_t)(mvx + (int)(uint32_t)(sx + x) * 8);
            const int16_t  row   = (int16_t)(mvy + (int)(uint32_t)(sy + y) * 8);
            const uint32_t cost  = cost0 + (uint32_t)mv_err_cost(row, col, p);
            if (cost < *best_cost) *best_cost = cost, *best_mvx = col, *best_mvy = row;
        }
    }
}
