/*
 * gen_golden_me.c — golden vectors for the open-loop ME SAD path (test infrastructure; never shipped).  Links the
 * REFERENCE's own C (EbMotionEstimation.c, EbComputeSAD_C.c compiled from /root/reference by oracle/ref.mk) and records
 * on deterministic SplitMix64 inputs:
 *   me_frame{n}   the full-pel search of every 64x64 block of an 8-bit frame against 2 references: the loop of
 *                 open_loop_me_fullpel_search_sblock (EbMotionEstimation.c:782-818, static there, restated here) over
 *                 the reference's svt_ext_all_sad_calculation_8x8_16x16_c + svt_ext_eight_sad_calculation_32x32_64x64_c
 *                 for groups of 8 positions and svt_ext_sad_calculation_8x8_16x16_c + _32x32_64x64_c for the rest of a
 *                 row (the 16x16 order of open_loop_me_get_search_point_results_block, :476-), best SADs reset to
 *                 MAX_SAD_VALUE first (:1363-1364); the reference pictures are padded by edge replication.
 *   all_sad / eight_sad / sad16 / sad32 / sad_loop
 *                 single calls of the five RTCD kernels on random blocks, random running bests.
 * usage: gen_golden_me <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "mcomp.h"
#include "golden_io.h"

void svt_pme_sad_loop_kernel_c(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                               uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                               uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                               int16_t search_position_start_x, int16_t search_position_start_y,
                               int16_t search_area_width, int16_t search_area_height, int16_t search_step, int16_t mvx,
                               int16_t mvy);

void svt_ext_all_sad_calculation_8x8_16x16_c(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                             uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                             uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                             uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                             Bool sub_sad);
void svt_ext_eight_sad_calculation_32x32_64x64_c(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                 uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                 uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]);
void svt_ext_sad_calculation_8x8_16x16_c(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                         uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                         uint32_t *p_best_mv16x16, uint32_t mv, uint32_t *p_sad16x16,
                                         uint32_t *p_sad8x8, Bool sub_sad);
void svt_ext_sad_calculation_32x32_64x64_c(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                           uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                           uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32);
void svt_sad_loop_kernel_c(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                           uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_search_center,
                           int16_t *y_search_center, uint32_t src_stride_raw, uint8_t skip_search_line,
                           int16_t search_area_width, int16_t search_area_height);

#define MAXSAD (128 * 128 * 255)
#define PAD 96

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* the 16x16 blocks in the order of the single-point path (EbMotionEstimation.c:476-...): raster in Z-order slots */
static const int kZ[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};

static void search_sb(uint8_t *src, int ss, uint8_t *refp, int rs, int ox, int oy, int saw, int sah, Bool sub,
                      uint32_t *best, uint32_t *bmv) {
    uint32_t *b8 = best, *b16 = best + 64, *b32 = best + 80, *b64 = best + 84;
    uint32_t *m8 = bmv, *m16 = bmv + 64, *m32 = bmv + 80, *m64 = bmv + 84;
    for (int k = 0; k < 85; k++) best[k] = MAXSAD, bmv[k] = 0;
    const int w8 = saw - (saw & 7);
    for (int y = 0; y < sah; y++) {
        for (int x = 0; x < w8; x += 8) {
            const uint32_t mv = ((uint32_t)(uint16_t)(oy + y) << 16) | (uint16_t)(ox + x);
            uint32_t       e16[16][8], e8[64][8], e32[4][8];
            svt_ext_all_sad_calculation_8x8_16x16_c(src, ss, refp + (size_t)y * rs + x, rs, mv, b8, b16, m8, m16, e16, e8,
                                                    sub);
            svt_ext_eight_sad_calculation_32x32_64x64_c(e16, b32, b64, m32, m64, mv, e32);
        }
        for (int x = w8; x < saw; x++) {
            const uint32_t mv = ((uint32_t)(uint16_t)(oy + y) << 16) | (uint16_t)(ox + x);
            uint32_t       s16[16], s8[4], s32[4];
            for (int by = 0; by < 4; by++)
                for (int bx = 0; bx < 4; bx++) {
                    const int q = kZ[4 * by + bx];
                    svt_ext_sad_calculation_8x8_16x16_c(src + 16 * by * ss + 16 * bx, ss,
                                                        refp + (size_t)(y + 16 * by) * rs + x + 16 * bx, rs, &b8[4 * q],
                                                        &b16[q], &m8[4 * q], &m16[q], mv, &s16[q], s8, sub);
                }
            svt_ext_sad_calculation_32x32_64x64_c(s16, b32, b64, m32, m64, mv, s32);
        }
    }
}

static void gen_frames(GoldenFile *g, Rng *r) {
    static const int cfg[][6] = {/* W, H, saw, sah, sub, origin span */
                                 {192, 128, 16, 16, 0, 40}, {128, 192, 13, 5, 1, 24}, {256, 128, 37, 9, 0, 120},
                                 {128, 128, 8, 1, 1, 8},    {192, 64, 1, 1, 0, 64},   {128, 128, 64, 33, 0, 70}};
    const int ncfg = (int)(sizeof cfg / sizeof cfg[0]);
    int32_t   meta[32][6];
    for (int n = 0; n < ncfg; n++) {
        const int W = cfg[n][0], H = cfg[n][1], saw = cfg[n][2], sah = cfg[n][3], sub = cfg[n][4], span = cfg[n][5];
        const int nref = 2, nsbx = W / 64, nsby = H / 64, nsb = nsbx * nsby;
        uint8_t  *src = malloc((size_t)W * H), *ref[2];
        for (int k = 0; k < W * H; k++) src[k] = 0; /* smooth content + noise, shifted copies as references */
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++)
                src[y * W + x] = (uint8_t)clampi(128 + (x * 3 + y * 2) % 97 - 48 + (int)rng_below(r, 17) - 8, 0, 255);
        const int PW = W + 2 * PAD, PH = H + 2 * PAD;
        uint8_t  *pad[2];
        for (int q = 0; q < nref; q++) {
            ref[q] = malloc((size_t)W * H);
            const int dx = (int)rng_below(r, 9) - 4, dy = (int)rng_below(r, 9) - 4;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++)
                    ref[q][y * W + x] = (uint8_t)clampi(src[clampi(y + dy, 0, H - 1) * W + clampi(x + dx, 0, W - 1)] +
                                                            (int)rng_below(r, 9) - 4,
                                                        0, 255);
            pad[q] = malloc((size_t)PW * PH); /* edge-replicated padding (svt_aom_generate_padding) */
            for (int y = 0; y < PH; y++)
                for (int x = 0; x < PW; x++)
                    pad[q][(size_t)y * PW + x] = ref[q][clampi(y - PAD, 0, H - 1) * W + clampi(x - PAD, 0, W - 1)];
        }
        int16_t  *org  = malloc(sizeof(int16_t) * nsb * nref * 2);
        uint32_t *best = malloc(sizeof(uint32_t) * nsb * nref * 85), *bmv = malloc(sizeof(uint32_t) * nsb * nref * 85);
        for (int sb = 0; sb < nsb; sb++)
            for (int q = 0; q < nref; q++) {
                const int t = sb * nref + q;
                int       ox = (int)rng_below(r, 2 * span + 1) - span - saw / 2;
                int       oy = (int)rng_below(r, 2 * span + 1) - span - sah / 2;
                const int sx0 = 64 * (sb % nsbx), sy0 = 64 * (sb / nsbx);
                ox = clampi(ox, -PAD - sx0, W + PAD - 64 - saw - 8 - sx0); /* the window stays inside the padding */
                oy = clampi(oy, -PAD - sy0, H + PAD - 64 - sah - sy0);
                org[2 * t] = (int16_t)ox, org[2 * t + 1] = (int16_t)oy;
                search_sb(src + (size_t)sy0 * W + sx0, W, pad[q] + (size_t)(PAD + sy0 + oy) * PW + PAD + sx0 + ox, PW, ox,
                          oy, saw, sah, (Bool)sub, best + (size_t)t * 85, bmv + (size_t)t * 85);
            }
        char nm[32];
        snprintf(nm, sizeof nm, "src%d", n), golden_put2(g, nm, 'B', (uint32_t)H, (uint32_t)W, src);
        for (int q = 0; q < nref; q++) snprintf(nm, sizeof nm, "ref%d_%d", n, q), golden_put2(g, nm, 'B', (uint32_t)H, (uint32_t)W, ref[q]);
        snprintf(nm, sizeof nm, "origin%d", n), golden_put2(g, nm, 'h', (uint32_t)(nsb * nref), 2, org);
        snprintf(nm, sizeof nm, "best_sad%d", n), golden_put2(g, nm, 'I', (uint32_t)(nsb * nref), 85, best);
        snprintf(nm, sizeof nm, "best_mv%d", n), golden_put2(g, nm, 'I', (uint32_t)(nsb * nref), 85, bmv);
        meta[n][0] = W, meta[n][1] = H, meta[n][2] = saw, meta[n][3] = sah, meta[n][4] = sub, meta[n][5] = nref;
        free(src), free(org), free(best), free(bmv);
        for (int q = 0; q < nref; q++) free(ref[q]), free(pad[q]);
    }
    golden_put2(g, "frame_meta", 'i', (uint32_t)ncfg, 6, meta);
}

static void fill(Rng *r, uint8_t *p, size_t n, int base, int amp) {
    for (size_t k = 0; k < n; k++) p[k] = (uint8_t)clampi(base + (int)rng_below(r, 2 * amp + 1) - amp, 0, 255);
}

static void gen_calls(GoldenFile *g, Rng *r) {
    enum { N = 48 };
    /* all_sad + eight_sad: a 64x64 block, 71-column window; random running bests */
    uint8_t  *blk = malloc(64 * 80), *win = malloc(80 * 80);
    uint32_t  io[N][2][85], e16[N][16][8], e32[N][4][8], mvs[N][3];
    uint8_t  *srcs = malloc((size_t)N * 64 * 80), *wins = malloc((size_t)N * 80 * 80);
    for (int n = 0; n < N; n++) {
        const int base = (int)rng_below(r, 256);
        fill(r, blk, 64 * 80, base, 1 + (int)rng_below(r, 60));
        fill(r, win, 80 * 80, base, 1 + (int)rng_below(r, 60));
        memcpy(srcs + (size_t)n * 64 * 80, blk, 64 * 80), memcpy(wins + (size_t)n * 80 * 80, win, 80 * 80);
        const uint32_t mv = ((uint32_t)(uint16_t)(int16_t)((int)rng_below(r, 200) - 100) << 16) |
                            (uint16_t)(int16_t)((int)rng_below(r, 200) - 100);
        const Bool sub = (Bool)(n & 1);
        uint32_t   b[85], m[85], e8[64][8];
        for (int k = 0; k < 85; k++) b[k] = rng_below(r, 4) ? 200000u + rng_below(r, 100000) : rng_below(r, 6000),
                                   m[k] = (uint32_t)rng_next(r);
        memcpy(io[n][0], b, sizeof b), memcpy(io[n][1], m, sizeof m);
        svt_ext_all_sad_calculation_8x8_16x16_c(blk, 80, win, 80, mv, b, b + 64, m, m + 64, e16[n], e8, sub);
        svt_ext_eight_sad_calculation_32x32_64x64_c(e16[n], b + 80, b + 84, m + 80, m + 84, mv, e32[n]);
        mvs[n][0] = mv, mvs[n][1] = sub, mvs[n][2] = 0;
        char nm[32];
        snprintf(nm, sizeof nm, "all_out_sad%d", n), golden_put1(g, nm, 'I', 85, b);
        snprintf(nm, sizeof nm, "all_out_mv%d", n), golden_put1(g, nm, 'I', 85, m);
    }
    golden_put2(g, "all_src", 'B', N * 64, 80, srcs);
    golden_put2(g, "all_win", 'B', N * 80, 80, wins);
    golden_put2(g, "all_in", 'I', N * 2, 85, io);
    golden_put2(g, "all_e16", 'I', N * 16, 8, e16);
    golden_put2(g, "all_e32", 'I', N * 4, 8, e32);
    golden_put2(g, "all_mv", 'I', N, 3, mvs);
    /* sad_loop: block sizes incl. the 16x16 skip-line path, src_stride_raw != ref_stride */
    static const int bs[][2] = {{8, 8}, {16, 16}, {16, 8}, {32, 32}, {64, 64}, {16, 32}, {8, 16}, {64, 16}};
    int32_t          lmeta[N][10];
    for (int n = 0; n < N; n++) {
        const int bw = bs[n % 8][0], bh = bs[n % 8][1], saw = 1 + (int)rng_below(r, 40), sah = 1 + (int)rng_below(r, 24);
        const int ss = 80, rs = 112, srr = rs + (n % 3 == 2 ? 8 : 0), skip = (n / 8) & 1;
        uint8_t  *s  = malloc((size_t)ss * 64), *rf = malloc((size_t)rs * 100 + 512);
        const int base = (int)rng_below(r, 256);
        fill(r, s, (size_t)ss * 64, base, 30), fill(r, rf, (size_t)rs * 100 + 512, base, 30);
        uint64_t best = 0;
        int16_t  xc = -1, yc = -1;
        svt_sad_loop_kernel_c(s, ss, rf, rs, bh, bw, &best, &xc, &yc, srr, (uint8_t)skip, (int16_t)saw, (int16_t)sah);
        lmeta[n][0] = bw, lmeta[n][1] = bh, lmeta[n][2] = saw, lmeta[n][3] = sah, lmeta[n][4] = ss, lmeta[n][5] = rs;
        lmeta[n][6] = srr, lmeta[n][7] = skip, lmeta[n][8] = (int32_t)best, lmeta[n][9] = (xc & 0xFFFF) | (yc << 16);
        char nm[32];
        snprintf(nm, sizeof nm, "loop_src%d", n), golden_put1(g, nm, 'B', (uint32_t)ss * 64, s);
        snprintf(nm, sizeof nm, "loop_ref%d", n), golden_put1(g, nm, 'B', (uint32_t)(rs * 100 + 512), rf);
        free(s), free(rf);
    }
    golden_put2(g, "loop_meta", 'i', N, 10, lmeta);
    free(blk), free(win), free(srcs), free(wins);
}

/* svt_pme_sad_loop_kernel_c (EbProductCodingLoop.c:1801) with every MV cost type (mcomp.c:43-68) and random
 * entropy tables; the running best starts at a random value */
static void gen_pme(GoldenFile *g, Rng *r) {
    enum { N = 40, TAB = 2 * (1 << 14) + 1 };
    static int jc[4], tab[2][TAB];
    for (int k = 0; k < 4; k++) jc[k] = (int)rng_below(r, 2000);
    for (int c = 0; c < 2; c++)
        for (int k = 0; k < TAB; k++) tab[c][k] = 100 + (int)rng_below(r, 3000) + abs(k - (1 << 14)) / 4;
    golden_put1(g, "pme_jc", 'i', 4, jc);
    golden_put2(g, "pme_tab", 'i', 2, TAB, tab);
    int32_t meta[N][20];
    for (int n = 0; n < N; n++) {
        static const int bs[][2] = {{8, 8}, {16, 16}, {32, 16}, {16, 64}, {64, 64}, {128, 128}, {4, 16}, {24, 8}};
        const int bw = bs[n % 8][0], bh = bs[n % 8][1];
        const int saw = 1 + (int)rng_below(r, 48), sah = 1 + (int)rng_below(r, 20), step = 1 + (int)rng_below(r, 3);
        const int ss = 160, rs = 240, rows = sah + bh + 2;
        uint8_t  *s = malloc((size_t)ss * bh), *rf = malloc((size_t)rs * rows);
        const int base = (int)rng_below(r, 256);
        for (int k = 0; k < ss * bh; k++) s[k] = (uint8_t)clampi(base + (int)rng_below(r, 61) - 30, 0, 255);
        for (int k = 0; k < rs * rows; k++) rf[k] = (uint8_t)clampi(base + (int)rng_below(r, 61) - 30, 0, 255);
        MV             ref_mv = {(int16_t)((int)rng_below(r, 400) - 200), (int16_t)((int)rng_below(r, 400) - 200)};
        MV_COST_PARAMS p;
        memset(&p, 0, sizeof p);
        p.ref_mv       = &ref_mv;
        p.mv_cost_type = (MV_COST_TYPE)(n % 6);
        p.mvjcost      = jc;
        p.mvcost[0]    = tab[0] + (1 << 14), p.mvcost[1] = tab[1] + (1 << 14);
        p.error_per_bit = 1 + (int)rng_below(r, 400);
        const int16_t sx = (int16_t)((int)rng_below(r, 40) - 20), sy = (int16_t)((int)rng_below(r, 40) - 20);
        const int16_t mvx = (int16_t)((int)rng_below(r, 600) - 300), mvy = (int16_t)((int)rng_below(r, 600) - 300);
        uint32_t      best = rng_below(r, 3) ? 0xFFFFFFFFu : (uint32_t)rng_below(r, (uint32_t)(bw * bh * 30));
        int16_t       bx = 111, by = -111;
        meta[n][10] = (int32_t)best;
        svt_pme_sad_loop_kernel_c(&p, s, ss, rf, rs, bh, bw, &best, &bx, &by, sx, sy, (int16_t)saw, (int16_t)sah,
                                  (int16_t)step, mvx, mvy);
        int32_t *m = meta[n];
        m[0] = bw, m[1] = bh, m[2] = saw, m[3] = sah, m[4] = step, m[5] = ss, m[6] = rs, m[7] = rows;
        m[8] = ref_mv.row, m[9] = ref_mv.col, m[11] = (int32_t)p.mv_cost_type, m[12] = p.error_per_bit;
        m[13] = sx, m[14] = sy, m[15] = mvx, m[16] = mvy, m[17] = (int32_t)best, m[18] = bx, m[19] = by;
        char nm[32];
        snprintf(nm, sizeof nm, "pme_src%d", n), golden_put1(g, nm, 'B', (uint32_t)(ss * bh), s);
        snprintf(nm, sizeof nm, "pme_ref%d", n), golden_put1(g, nm, 'B', (uint32_t)(rs * rows), rf);
        free(s), free(rf);
    }
    golden_put2(g, "pme_meta", 'i', N, 20, meta);
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "tests/golden";
    char        path[512];
    snprintf(path, sizeof path, "%s/me_sad.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4D45534144000001ull};
    gen_frames(&g, &r);
    gen_calls(&g, &r);
    gen_pme(&g, &r);
    golden_close(&g);
    printf("wrote %s\n", path);
    return 0;
}
