/*
 * gen_golden_cdef.c — golden-vector generator (test infrastructure; never shipped).
 *
 * Links the REFERENCE's own C kernels (compiled from /root/reference by oracle/ref.mk) and records
 * their outputs on deterministic SplitMix64 inputs.  Sweeps mirror the reference's gtests
 * (test/CdefTest.cc: CDEFBlockTest :94-366, CDEFFindDirTest :435-497, ComputeCdefDistMatchTest
 * :760-961, SearchOneDualMatchTest :996-1070), with our own PRNG in place of std::mt19937.
 *
 * usage: gen_golden_cdef <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbCdef.h"
#include "common_dsp_rtcd.h"
#include "aom_dsp_rtcd.h"
#include "golden_io.h"

static void bind_c_kernels(void) {
    svt_cdef_filter_block       = svt_cdef_filter_block_c;
    svt_aom_cdef_find_dir       = svt_aom_cdef_find_dir_c;
    svt_aom_cdef_find_dir_dual  = svt_aom_cdef_find_dir_dual_c;
    svt_compute_cdef_dist_16bit = svt_aom_compute_cdef_dist_c;
    svt_compute_cdef_dist_8bit  = svt_aom_compute_cdef_dist_8bit_c;
    svt_search_one_dual         = svt_search_one_dual_c;
    svt_aom_copy_rect8_8bit_to_16bit = svt_aom_copy_rect8_8bit_to_16bit_c;
}

static uint16_t rnd_px(Rng *r, int bd, int level, int bits) {
    int v = (int)(rng_next(r) & ((1u << bits) - 1)) + level;
    int m = (1 << bd) - 1;
    return (uint16_t)(v < 0 ? 0 : v > m ? m : v);
}

/* ---- find_dir: 8x8 blocks, bd 8/10/12 ---- */
static void gen_find_dir(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/cdef_find_dir.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x5EED0001ull};
    enum { N = 600 };
    static uint16_t img[N][64];
    static int32_t  var[N], bdv[N];
    static uint8_t  dirs[N];
    for (int n = 0; n < N; n++) {
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12;
        const int kind = (n / 3) % 3;
        if (kind == 0) { /* CDEFFindDirTest-style random */
            const int bits = 1 + rng_below(&r, bd), level = rng_below(&r, 1 << bd);
            for (int i = 0; i < 64; i++) img[n][i] = rnd_px(&r, bd, level - (1 << (bits - 1)), bits);
        } else { /* oriented ramps so every direction wins somewhere */
            const int dy = (int)rng_below(&r, 9) - 4, dx = (int)rng_below(&r, 9) - 4;
            const int base = rng_below(&r, 1 << bd), amp = 1 + rng_below(&r, 1 << (bd - 3));
            for (int i = 0; i < 64; i++) {
                int v = base + amp * ((i / 8) * dy + (i % 8) * dx) / 4 + (int)rng_below(&r, 1 + (kind == 2 ? amp : 0));
                img[n][i] = (uint16_t)(v < 0 ? 0 : v >= (1 << bd) ? (1 << bd) - 1 : v);
            }
        }
        bdv[n]  = bd;
        dirs[n] = svt_aom_cdef_find_dir_c(img[n], 8, &var[n], bd - 8);
    }
    golden_put2(&g, "img", 'H', N, 64, img);
    golden_put1(&g, "bd", 'i', N, bdv);
    golden_put1(&g, "var", 'i', N, var);
    golden_put1(&g, "dir", 'B', N, dirs);
    golden_close(&g);
}

/* ---- filter_block: all bsizes, 16 boundary masks, bd 8/10/12, strengths/dirs/damping ---- */
#define FB_WIN 12 /* rows -2..9, cols -2..9 around the block origin */
static void gen_filter_block(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/cdef_filter_block.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x5EED0002ull};
    enum { N = 3000 };
    static uint16_t win[N][FB_WIN * FB_WIN];
    static int32_t  prm[N][10]; /* bd, bsize, pri, sec, dir, pdamp, sdamp, ss, use8, boundary */
    static uint16_t out[N][64];
    static uint16_t inbuf[CDEF_INBUF_SIZE];
    for (int n = 0; n < N; n++) {
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12, cs = bd - 8;
        const int bsize = (n / 3) % 4; /* BLOCK_4X4..BLOCK_8X8 */
        const int boundary = rng_below(&r, 16);
        const int bits = 1 + rng_below(&r, bd), level = rng_below(&r, 1 << bd);
        for (int i = 0; i < CDEF_INBUF_SIZE; i++) inbuf[i] = rnd_px(&r, bd, level, bits);
        uint16_t *in = inbuf + CDEF_VBORDER * CDEF_BSTRIDE + CDEF_HBORDER;
        const int bh = (bsize == BLOCK_8X8 || bsize == BLOCK_4X8) ? 8 : 4;
        const int bw = (bsize == BLOCK_8X8 || bsize == BLOCK_8X4) ? 8 : 4;
        for (int i = -3; i < bh + 3; i++)
            for (int j = -8; j < bw + 8; j++) {
                const int large = ((boundary & 1) && j < 0) || ((boundary & 2) && j >= bw) ||
                    ((boundary & 4) && i < 0) || ((boundary & 8) && i >= bh);
                if (large)
                    in[i * CDEF_BSTRIDE + j] = CDEF_VERY_LARGE;
            }
        int pri = rng_below(&r, 20);
        pri     = pri >= 16 ? 19 : pri; /* CdefTest.cc:160-163 includes 19 */
        pri <<= cs;
        if (rng_below(&r, 4) == 0) /* adjusted luma strengths are arbitrary in [0, pri] */
            pri = rng_below(&r, (15 << cs) + 1);
        static const int secs[4] = {0, 1, 2, 4};
        const int        sec = secs[rng_below(&r, 4)] << cs;
        const int        d   = rng_below(&r, 8);
        const int pdamp = 3 + cs + rng_below(&r, 4) - (rng_below(&r, 3) == 0);
        const int sdamp = 3 + cs + rng_below(&r, 4) - (rng_below(&r, 3) == 0);
        const int ss = bsize == BLOCK_4X4 ? 1 : 1 + rng_below(&r, 2);
        const int use8 = bd == 8 && rng_below(&r, 2);
        for (int i = 0; i < FB_WIN; i++)
            for (int j = 0; j < FB_WIN; j++) win[n][i * FB_WIN + j] = in[(i - 2) * CDEF_BSTRIDE + (j - 2)];
        uint8_t  d8[64];
        uint16_t d16[64];
        memset(d8, 0xA5, sizeof d8);
        for (int i = 0; i < 64; i++) d16[i] = 0xA5A5;
        svt_cdef_filter_block_c(use8 ? d8 : NULL, use8 ? NULL : d16, bw, in, pri, sec, d, pdamp, sdamp, bsize, cs,
                                (uint8_t)ss);
        for (int i = 0; i < 64; i++) out[n][i] = use8 ? d8[i] : d16[i];
        int32_t p[10] = {bd, bsize, pri, sec, d, pdamp, sdamp, ss, use8, boundary};
        memcpy(prm[n], p, sizeof p);
    }
    golden_put2(&g, "win", 'H', N, FB_WIN * FB_WIN, win);
    golden_put2(&g, "params", 'i', N, 10, prm);
    golden_put2(&g, "out", 'H', N, 64, out);
    golden_close(&g);
}

/* ---- compute_cdef_dist (8bit & 16bit): random dlists, planes, bsizes, subsampling ---- */
static void gen_cdef_dist(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/cdef_dist.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x5EED0003ull};
    enum { N = 120, ST = 68 };
    static uint16_t srcs[N][64 * ST];  /* source block region (stride ST) */
    static uint16_t flt[N][64 * 64];   /* packed filtered blocks */
    static uint8_t  dl[N][64][2];
    static int32_t  prm[N][6]; /* bd, bsize, count, pli, ss, is8 */
    static uint64_t res[N];
    for (int n = 0; n < N; n++) {
        const int bd = n % 2 ? 10 : 8, cs = bd - 8;
        const int is8 = bd == 8 && (n / 2) % 2;
        const int bsize = rng_below(&r, 4);
        const int pli = bsize == BLOCK_8X8 ? (int)rng_below(&r, 2) : 1;
        const int lbh = (bsize == BLOCK_8X8 || bsize == BLOCK_4X8) ? 3 : 2;
        const int lbw = (bsize == BLOCK_8X8 || bsize == BLOCK_8X4) ? 3 : 2;
        int ss = 1 + rng_below(&r, 4);
        ss     = ss == 3 ? 4 : ss;
        if (bsize == BLOCK_4X4) ss = 1;
        else if (bsize != BLOCK_8X8 && ss > 2) ss = 2;
        /* unique random block positions within an 8x8 grid of blocks */
        uint8_t used[64] = {0};
        const int count = 1 + rng_below(&r, 64);
        for (int i = 0; i < count; i++) {
            int p;
            do p = rng_below(&r, 64);
            while (used[p]);
            used[p]  = 1;
            dl[n][i][0] = (uint8_t)(p / 8);
            dl[n][i][1] = (uint8_t)(p % 8);
        }
        const int level = rng_below(&r, 1 << bd), bits = 1 + rng_below(&r, bd);
        for (int i = 0; i < 64 * ST; i++) srcs[n][i] = rnd_px(&r, bd, level, bits);
        for (int i = 0; i < 64 * 64; i++) {
            int v = rng_below(&r, 3) ? srcs[n][rng_below(&r, 64 * ST)] : rnd_px(&r, bd, level, bits);
            flt[n][i] = (uint16_t)v;
        }
        CdefList list[64];
        for (int i = 0; i < count; i++) {
            list[i].by = dl[n][i][0];
            list[i].bx = dl[n][i][1];
        }
        (void)lbh;
        (void)lbw;
        if (is8) {
            static uint8_t s8[64 * ST], f8[64 * 64];
            for (int i = 0; i < 64 * ST; i++) s8[i] = (uint8_t)srcs[n][i];
            for (int i = 0; i < 64 * 64; i++) f8[i] = (uint8_t)flt[n][i];
            res[n] = svt_aom_compute_cdef_dist_8bit_c(s8, ST, f8, list, count, bsize, cs, pli, (uint8_t)ss);
        } else
            res[n] = svt_aom_compute_cdef_dist_c(srcs[n], ST, flt[n], list, count, bsize, cs, pli, (uint8_t)ss);
        int32_t p[6] = {bd, bsize, count, pli, ss, is8};
        memcpy(prm[n], p, sizeof p);
    }
    golden_put2(&g, "src", 'H', N, 64 * ST, srcs);
    golden_put2(&g, "flt", 'H', N, 64 * 64, flt);
    golden_put2(&g, "dlist", 'B', N, 128, dl);
    golden_put2(&g, "params", 'i', N, 6, prm);
    golden_put1(&g, "dist", 'Q', N, res);
    golden_close(&g);
}

/* ---- search_one_dual: sb_count 100, nb 0..7 preselected, end_gi 64 (SearchOneDualMatchTest) ---- */
static void gen_search_one_dual(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/cdef_search_one_dual.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x5EED0004ull};
    enum { N = 12, SB = 100 };
    static uint64_t mse[N][2][SB][64];
    static int32_t  lev[N][2][16], lev_out[N][2][16], prm[N][3];
    static uint64_t res[N];
    for (int n = 0; n < N; n++) {
        const int nb = n % 8, start = n >= 8 ? (int)rng_below(&r, 8) : 0, end = n >= 10 ? 32 + rng_below(&r, 33) : 64;
        for (int p = 0; p < 2; p++)
            for (int s = 0; s < SB; s++)
                for (int k = 0; k < 64; k++) {
                    /* mixture of realistic magnitudes and forced ties */
                    uint64_t v = rng_next(&r) % (n % 3 == 0 ? 1000u : (1u << 30));
                    mse[n][p][s][k] = v;
                }
        for (int i = 0; i < 16; i++) {
            lev[n][0][i] = rng_below(&r, 64);
            lev[n][1][i] = rng_below(&r, 64);
        }
        uint64_t *rows0[SB], *rows1[SB];
        for (int s = 0; s < SB; s++) {
            rows0[s] = mse[n][0][s];
            rows1[s] = mse[n][1][s];
        }
        uint64_t **m[2] = {rows0, rows1};
        memcpy(lev_out[n], lev[n], sizeof lev[n]);
        res[n] = svt_search_one_dual_c(lev_out[n][0], lev_out[n][1], nb, m, SB, start, end);
        prm[n][0] = nb;
        prm[n][1] = start;
        prm[n][2] = end;
    }
    golden_put(&g, "mse", 'Q', 4, (uint32_t[]){N, 2, SB, 64}, mse);
    golden_put(&g, "lev_in", 'i', 3, (uint32_t[]){N, 2, 16}, lev);
    golden_put(&g, "lev_out", 'i', 3, (uint32_t[]){N, 2, 16}, lev_out);
    golden_put2(&g, "params", 'i', N, 3, prm);
    golden_put1(&g, "best", 'Q', N, res);
    golden_close(&g);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    bind_c_kernels();
    gen_find_dir(argv[1]);
    gen_filter_block(argv[1]);
    gen_cdef_dist(argv[1]);
    gen_search_one_dual(argv[1]);
    printf("cdef golden vectors written to %s\n", argv[1]);
    return 0;
}
