/*
 * gen_golden_frame.c — golden vectors for the frame-buffer work around the path (test infrastructure; never shipped).
 * Links the REFERENCE's own C (EbPackUnPack_C.c, EbMcp.c, EbRestoration.c compiled from /root/reference by
 * oracle/ref.mk) and records on deterministic SplitMix64 planes with odd sizes and strides:
 *   conv{n}   svt_convert_8bit_to_16bit_c / svt_convert_16bit_to_8bit_c (EbPackUnPack_C.c:270-283)
 *   pad{n}    svt_aom_generate_padding / svt_aom_generate_padding16_bit (EbMcp.c:95-150, 201-240)
 *   ext{n}    svt_extend_frame (EbRestoration.c:197-203), low and high bit depth
 * Each record holds the whole buffer before and after the call (the samples the call must leave alone included).
 * usage: gen_golden_frame <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "common_dsp_rtcd.h"
#include "golden_io.h"

void svt_convert_8bit_to_16bit_c(uint8_t *src, uint32_t src_stride, uint16_t *dst, uint32_t dst_stride, uint32_t width,
                                 uint32_t height);
void svt_convert_16bit_to_8bit_c(uint16_t *src, uint32_t src_stride, uint8_t *dst, uint32_t dst_stride, uint32_t width,
                                 uint32_t height);
void svt_aom_generate_padding(EbByte src_pic, uint32_t src_stride, uint32_t original_src_width,
                              uint32_t original_src_height, uint32_t padding_width, uint32_t padding_height);
void svt_aom_generate_padding16_bit(uint16_t *src_pic, uint32_t src_stride, uint32_t original_src_width,
                                    uint32_t original_src_height, uint32_t padding_width, uint32_t padding_height);
void svt_extend_frame(uint8_t *data, int32_t width, int32_t height, int32_t stride, int32_t border_horz,
                      int32_t border_vert, int32_t highbd);

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "tests/golden";
    char        path[512], nm[32];
    snprintf(path, sizeof path, "%s/frame_ops.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4652414D45000001ull};
    svt_memcpy = svt_memcpy_c;
    enum { N = 12 };
    int32_t meta[3][N][8] = {{{0}}}; /* fields a case does not use stay 0: the fixture is reproducible */
    for (int n = 0; n < N; n++) {
        /* conversion: w x h inside strides with slack; the destination's slack keeps its old contents */
        const int w = 1 + (int)rng_below(&r, 200), h = 1 + (int)rng_below(&r, 40);
        const int ss = w + (int)rng_below(&r, 40), ds = w + (int)rng_below(&r, 40), dir16 = n & 1;
        const size_t ns = (size_t)ss * h, nd = (size_t)ds * h;
        if (!dir16) { /* 8 -> 16 */
            uint8_t  *s = malloc(ns);
            uint16_t *d = malloc(2 * nd), *d0 = malloc(2 * nd);
            for (size_t k = 0; k < ns; k++) s[k] = (uint8_t)rng_next(&r);
            for (size_t k = 0; k < nd; k++) d[k] = d0[k] = (uint16_t)rng_next(&r);
            svt_convert_8bit_to_16bit_c(s, ss, d, ds, w, h);
            snprintf(nm, sizeof nm, "conv_src%d", n), golden_put1(&g, nm, 'B', (uint32_t)ns, s);
            snprintf(nm, sizeof nm, "conv_dst0_%d", n), golden_put1(&g, nm, 'H', (uint32_t)nd, d0);
            snprintf(nm, sizeof nm, "conv_dst%d", n), golden_put1(&g, nm, 'H', (uint32_t)nd, d);
            free(s), free(d), free(d0);
        } else { /* 16 -> 8 */
            uint16_t *s = malloc(2 * ns);
            uint8_t  *d = malloc(nd), *d0 = malloc(nd);
            for (size_t k = 0; k < ns; k++) s[k] = (uint16_t)rng_next(&r);
            for (size_t k = 0; k < nd; k++) d[k] = d0[k] = (uint8_t)rng_next(&r);
            svt_convert_16bit_to_8bit_c(s, ss, d, ds, w, h);
            snprintf(nm, sizeof nm, "conv_src%d", n), golden_put1(&g, nm, 'H', (uint32_t)ns, s);
            snprintf(nm, sizeof nm, "conv_dst0_%d", n), golden_put1(&g, nm, 'B', (uint32_t)nd, d0);
            snprintf(nm, sizeof nm, "conv_dst%d", n), golden_put1(&g, nm, 'B', (uint32_t)nd, d);
            free(s), free(d), free(d0);
        }
        meta[0][n][0] = w, meta[0][n][1] = h, meta[0][n][2] = ss, meta[0][n][3] = ds, meta[0][n][4] = dir16;
        /* padding: a (h + 2 ph) x stride buffer, visible area at (pw, ph), stride slack beyond w + 2 pw */
        {
            const int w2 = 1 + (int)rng_below(&r, 150), h2 = 1 + (int)rng_below(&r, 30);
            const int pw = (int)rng_below(&r, 40), ph = (int)rng_below(&r, 20), st = w2 + 2 * pw + (int)rng_below(&r, 24);
            const int hb = n & 1;
            const size_t nb = (size_t)st * (h2 + 2 * ph);
            if (hb) {
                uint16_t *b = malloc(2 * nb), *b0 = malloc(2 * nb);
                for (size_t k = 0; k < nb; k++) b[k] = b0[k] = (uint16_t)(rng_next(&r) & 1023);
                svt_aom_generate_padding16_bit(b, st, w2, h2, pw, ph);
                snprintf(nm, sizeof nm, "pad_in%d", n), golden_put1(&g, nm, 'H', (uint32_t)nb, b0);
                snprintf(nm, sizeof nm, "pad_out%d", n), golden_put1(&g, nm, 'H', (uint32_t)nb, b);
                free(b), free(b0);
            } else {
                uint8_t *b = malloc(nb), *b0 = malloc(nb);
                for (size_t k = 0; k < nb; k++) b[k] = b0[k] = (uint8_t)rng_next(&r);
                svt_aom_generate_padding(b, st, w2, h2, pw, ph);
                snprintf(nm, sizeof nm, "pad_in%d", n), golden_put1(&g, nm, 'B', (uint32_t)nb, b0);
                snprintf(nm, sizeof nm, "pad_out%d", n), golden_put1(&g, nm, 'B', (uint32_t)nb, b);
                free(b), free(b0);
            }
            meta[1][n][0] = w2, meta[1][n][1] = h2, meta[1][n][2] = st, meta[1][n][3] = pw, meta[1][n][4] = ph,
            meta[1][n][5] = hb;
        }
        /* extension: visible area at (bh + off, bv) of a buffer with extra slack on every side */
        {
            const int w3 = 1 + (int)rng_below(&r, 150), h3 = 1 + (int)rng_below(&r, 30);
            const int bh = (int)rng_below(&r, 40), bv = (int)rng_below(&r, 20), slack = 1 + (int)rng_below(&r, 9);
            const int st = w3 + 2 * bh + 2 * slack, rows = h3 + 2 * bv + 2;
            const int hb = (n >> 1) & 1;
            const size_t nb = (size_t)st * rows, o = (size_t)(bv + 1) * st + bh + slack;
            if (hb) {
                uint16_t *b = malloc(2 * nb), *b0 = malloc(2 * nb);
                for (size_t k = 0; k < nb; k++) b[k] = b0[k] = (uint16_t)(rng_next(&r) & 1023);
                svt_extend_frame(CONVERT_TO_BYTEPTR(b + o), w3, h3, st, bh, bv, 1);
                snprintf(nm, sizeof nm, "ext_in%d", n), golden_put1(&g, nm, 'H', (uint32_t)nb, b0);
                snprintf(nm, sizeof nm, "ext_out%d", n), golden_put1(&g, nm, 'H', (uint32_t)nb, b);
                free(b), free(b0);
            } else {
                uint8_t *b = malloc(nb), *b0 = malloc(nb);
                for (size_t k = 0; k < nb; k++) b[k] = b0[k] = (uint8_t)rng_next(&r);
                svt_extend_frame(b + o, w3, h3, st, bh, bv, 0);
                snprintf(nm, sizeof nm, "ext_in%d", n), golden_put1(&g, nm, 'B', (uint32_t)nb, b0);
                snprintf(nm, sizeof nm, "ext_out%d", n), golden_put1(&g, nm, 'B', (uint32_t)nb, b);
                free(b), free(b0);
            }
            meta[2][n][0] = w3, meta[2][n][1] = h3, meta[2][n][2] = st, meta[2][n][3] = bh, meta[2][n][4] = bv,
            meta[2][n][5] = hb, meta[2][n][6] = (int32_t)o;
        }
    }
    uint32_t dims[3] = {3, N, 8};
    golden_put(&g, "meta", 'i', 3, dims, meta);
    golden_close(&g);
    printf("wrote %s\n", path);
    return 0;
}
