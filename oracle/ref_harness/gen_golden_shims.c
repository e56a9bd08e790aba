/*
 * gen_golden_shims.c — golden vectors for the per-block RTCD shims added in round 2 (test infrastructure; never
 * shipped).  Links the REFERENCE's own C (and, for the AVX2-only svt_cdef_filter_block_8xn_16, its AVX2 source),
 * compiled from /root/reference by oracle/ref.mk, and records on deterministic SplitMix64 inputs:
 *   proj_error / proj_subspace  svt_av1_{lowbd,highbd}_pixel_proj_error_c, svt_get_proj_subspace_c on flt0/flt1
 *                               from svt_av1_selfguided_restoration_c, every ep (incl. r = 0 ones), random xq
 *   subpel_var                  svt_aom_sub_pixel_variance{W}x{H}_c for the 22 sizes x every (xoffset, yoffset)
 *   mse / var_highbd / nxm_sad  svt_aom_mse16x16_c, svt_aom_highbd_8_mse16x16_c, svt_aom_variance_highbd_c,
 *                               svt_fast_loop_nxm_sad_kernel (the C nxm and nxm_sub_sampled entries)
 *   cdef_8xn / copy_rect8       svt_cdef_filter_block_8xn_16_avx2 (ss 1/2/4), svt_aom_copy_rect8_8bit_to_16bit_c
 * usage: gen_golden_shims <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "EbRestoration.h"
#include "EbCdef.h"
#include "common_dsp_rtcd.h"
#include "aom_dsp_rtcd.h"
#include "golden_io.h"

void     svt_cdef_filter_block_8xn_16_avx2(const uint16_t *const in, const int32_t pri_strength,
                                           const int32_t sec_strength, const int32_t dir, int32_t pri_damping,
                                           int32_t sec_damping, const int32_t coeff_shift, uint16_t *const dst,
                                           const int32_t dstride, uint8_t height, uint8_t subsampling_factor);
uint32_t svt_fast_loop_nxm_sad_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                      uint32_t ref_stride, uint32_t height, uint32_t width);

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* ------------------------------------------------------------------------------------------- */
#define PN 64
static void gen_proj(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/lr_proj.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x50524F4A00000001ull};
    /* per case: meta {bd, w, h, eps, xq0, xq1, err, sub_xq0, sub_xq1}; src / dat (h x w, stride w), flt0 / flt1 */
    int32_t *meta = calloc(PN, 9 * sizeof(int32_t));
    int32_t *tmp  = malloc(RESTORATION_UNITPELS_MAX * 2 * sizeof(int32_t));
    for (int n = 0; n < PN; n++) {
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12, hbd = bd > 8, maxv = (1 << bd) - 1;
        const int w = 8 + (int)rng_below(&r, 57), h = 8 + (int)rng_below(&r, 57), eps = n % 16; /* <= a 64x64 processing unit */
        const int st = w + 6;
        uint16_t *in  = malloc(sizeof(uint16_t) * (size_t)(h + 6) * st);
        uint16_t *src = malloc(sizeof(uint16_t) * (size_t)w * h), *dat = malloc(sizeof(uint16_t) * (size_t)w * h);
        const int base = (int)rng_below(&r, (uint32_t)maxv + 1), amp = 1 + (int)rng_below(&r, (uint32_t)(maxv / 4 + 1));
        for (int k = 0; k < (h + 6) * st; k++) in[k] = (uint16_t)clampi(base + (int)rng_below(&r, 2 * amp + 1) - amp, 0, maxv);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                dat[y * w + x] = in[(y + 3) * st + x + 3];
                src[y * w + x] = (uint16_t)clampi(dat[y * w + x] + (int)rng_below(&r, 2 * (8 << (bd - 8)) + 1) - (8 << (bd - 8)), 0, maxv);
            }
        int32_t *f0 = calloc((size_t)w * h, sizeof(int32_t)), *f1 = calloc((size_t)w * h, sizeof(int32_t)); /* r = 0 eps leave one unwritten */
        uint8_t *in8 = malloc((size_t)(h + 6) * st), *src8 = malloc((size_t)w * h), *dat8 = malloc((size_t)w * h);
        for (int k = 0; k < (h + 6) * st; k++) in8[k] = (uint8_t)in[k];
        for (int k = 0; k < w * h; k++) src8[k] = (uint8_t)src[k], dat8[k] = (uint8_t)dat[k];
        const uint8_t *ip = hbd ? CONVERT_TO_BYTEPTR(in + 3 * st + 3) : in8 + 3 * st + 3;
        svt_av1_selfguided_restoration_c(ip, w, h, st, f0, f1, w, eps, bd, hbd);
        const SgrParamsType *prm = &svt_aom_eb_sgr_params[eps];
        int32_t              xq[2] = {-96 + (int)rng_below(&r, 192), -64 + (int)rng_below(&r, 192)};
        if (prm->r[0] == 0) xq[0] = 0;
        if (prm->r[1] == 0) xq[1] = 0;
        const uint8_t *sp = hbd ? CONVERT_TO_BYTEPTR(src) : src8, *dp = hbd ? CONVERT_TO_BYTEPTR(dat) : dat8;
        const int64_t  err = hbd ? svt_av1_highbd_pixel_proj_error_c(sp, w, h, w, dp, w, f0, w, f1, w, xq, prm)
                                 : svt_av1_lowbd_pixel_proj_error_c(sp, w, h, w, dp, w, f0, w, f1, w, xq, prm);
        int32_t sxq[2];
        svt_get_proj_subspace_c(sp, w, h, w, dp, w, hbd, f0, w, f1, w, sxq, prm);
        int32_t *m = meta + 9 * n;
        m[0] = bd, m[1] = w, m[2] = h, m[3] = eps, m[4] = xq[0], m[5] = xq[1], m[6] = (int32_t)err, m[7] = sxq[0], m[8] = sxq[1];
        if ((int64_t)m[6] != err) fprintf(stderr, "proj error overflows int32 at case %d\n", n), exit(1);
        char nm[32];
        snprintf(nm, sizeof nm, "src%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)h, (uint32_t)w, src);
        snprintf(nm, sizeof nm, "dat%d", n);
        golden_put2(&g, nm, 'H', (uint32_t)h, (uint32_t)w, dat);
        snprintf(nm, sizeof nm, "flt0_%d", n);
        golden_put2(&g, nm, 'i', (uint32_t)h, (uint32_t)w, f0);
        snprintf(nm, sizeof nm, "flt1_%d", n);
        golden_put2(&g, nm, 'i', (uint32_t)h, (uint32_t)w, f1);
        free(in), free(src), free(dat), free(f0), free(f1), free(in8), free(src8), free(dat8);
    }
    golden_put2(&g, "meta", 'i', PN, 9, meta);
    int32_t sgr[16 * 4];
    for (int e = 0; e < 16; e++)
        for (int k = 0; k < 2; k++) sgr[4 * e + k] = svt_aom_eb_sgr_params[e].r[k], sgr[4 * e + 2 + k] = svt_aom_eb_sgr_params[e].s[k];
    golden_put2(&g, "sgr_params", 'i', 16, 4, sgr);
    golden_close(&g);
    free(meta), free(tmp);
}

/* ------------------------------------------------------------------------------------------- */
typedef uint32_t (*SubpelFn)(const uint8_t *, int, int, int, const uint8_t *, int, uint32_t *);
static const int SW[22] = {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 64, 128, 128, 4, 16, 8, 32, 16, 64};
static const int SH[22] = {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 128, 64, 128, 16, 4, 32, 8, 64, 16};
static const SubpelFn SUBPEL[22] = {
    svt_aom_sub_pixel_variance4x4_c,    svt_aom_sub_pixel_variance4x8_c,    svt_aom_sub_pixel_variance8x4_c,
    svt_aom_sub_pixel_variance8x8_c,    svt_aom_sub_pixel_variance8x16_c,   svt_aom_sub_pixel_variance16x8_c,
    svt_aom_sub_pixel_variance16x16_c,  svt_aom_sub_pixel_variance16x32_c,  svt_aom_sub_pixel_variance32x16_c,
    svt_aom_sub_pixel_variance32x32_c,  svt_aom_sub_pixel_variance32x64_c,  svt_aom_sub_pixel_variance64x32_c,
    svt_aom_sub_pixel_variance64x64_c,  svt_aom_sub_pixel_variance64x128_c, svt_aom_sub_pixel_variance128x64_c,
    svt_aom_sub_pixel_variance128x128_c, svt_aom_sub_pixel_variance4x16_c,  svt_aom_sub_pixel_variance16x4_c,
    svt_aom_sub_pixel_variance8x32_c,   svt_aom_sub_pixel_variance32x8_c,   svt_aom_sub_pixel_variance16x64_c,
    svt_aom_sub_pixel_variance64x16_c};

static void gen_md(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/md_shims.bin", dir);
    GoldenFile g  = golden_open(path);
    Rng        r  = {0x4D44534800000001ull};
    /* four shared buffer pairs (mode 0 random, 1 near, 2 max difference, 3 equal), 8-bit and 16-bit (10/12-bit
     * values), 192 x 192; each case reads a block at an offset of one of them */
    enum { S = 192 };
    uint8_t  *A = malloc(4 * S * S), *B = malloc(4 * S * S);
    uint16_t *A16 = malloc(2 * 4 * S * S), *B16 = malloc(2 * 4 * S * S);
    for (int m = 0; m < 4; m++)
        for (int k = 0; k < S * S; k++) {
            const int bd = 10 + 2 * (m & 1), v8 = (int)rng_below(&r, 256), v16 = (int)rng_below(&r, 1u << bd);
            uint8_t  *pa = A + m * S * S, *pb = B + m * S * S;
            uint16_t *qa = A16 + m * S * S, *qb = B16 + m * S * S;
            pa[k] = (uint8_t)v8, qa[k] = (uint16_t)v16;
            pb[k] = m == 0 ? (uint8_t)rng_below(&r, 256) : m == 1 ? (uint8_t)clampi(v8 + (int)rng_below(&r, 9) - 4, 0, 255)
                  : m == 2 ? (uint8_t)(255 - v8) : (uint8_t)v8;
            qb[k] = m == 0 ? (uint16_t)rng_below(&r, 1u << bd)
                  : m == 1 ? (uint16_t)clampi(v16 + (int)rng_below(&r, 33) - 16, 0, (1 << bd) - 1)
                  : m == 2 ? (uint16_t)(((1 << bd) - 1) - v16) : (uint16_t)v16;
        }
    uint32_t d3[3] = {4, S, S};
    golden_put(&g, "A", 'B', 3, d3, A);
    golden_put(&g, "B", 'B', 3, d3, B);
    golden_put(&g, "A16", 'H', 3, d3, A16);
    golden_put(&g, "B16", 'H', 3, d3, B16);
    /* sub-pixel variance: the 22 sizes x 64 (xoffset, yoffset) x 4 buffer pairs at offset (m, 3m) */
    for (int s = 0; s < 22; s++) {
        uint32_t res[4 * 64 * 2];
        for (int m = 0; m < 4; m++)
            for (int o = 0; o < 64; o++) {
                uint32_t       sse;
                const uint8_t *a = A + m * S * S + m * S + 3 * m, *b = B + m * S * S + m * S + 3 * m;
                res[(m * 64 + o) * 2]     = SUBPEL[s](a, S, o & 7, o >> 3, b, S, &sse);
                res[(m * 64 + o) * 2 + 1] = sse;
            }
        char nm[32];
        snprintf(nm, sizeof nm, "spv%d", s);
        golden_put2(&g, nm, 'I', 4 * 64, 2, res);
    }
    /* mse16x16 / highbd_8_mse16x16 / variance_highbd (any w x h up to 128) / nxm SAD, 400 cases:
     * meta {mode, oy, ox, w, h}, res {mse, sse, hbd8 sse, var_highbd, its sse, nxm sad} */
    const int N    = 400;
    int32_t  *meta = calloc(N, 5 * sizeof(int32_t));
    uint32_t *res  = calloc(N, 6 * sizeof(uint32_t));
    for (int n = 0; n < N; n++) {
        const int m = n % 4, oy = (int)rng_below(&r, 64), ox = (int)rng_below(&r, 64);
        const int w = 1 + (int)rng_below(&r, 128), h = 1 + (int)rng_below(&r, 128);
        const uint8_t  *pa = A + m * S * S + oy * S + ox, *pb = B + m * S * S + oy * S + ox;
        uint16_t       *qa = A16 + m * S * S + oy * S + ox, *qb = B16 + m * S * S + oy * S + ox;
        uint32_t        sse;
        res[6 * n + 0] = svt_aom_mse16x16_c(pa, S, pb, S, &sse);
        res[6 * n + 1] = sse;
        svt_aom_highbd_8_mse16x16_c(CONVERT_TO_BYTEPTR(qa), S, CONVERT_TO_BYTEPTR(qb), S, &sse);
        res[6 * n + 2] = sse;
        res[6 * n + 3] = svt_aom_variance_highbd_c(qa, S, qb, S, w, h, &sse);
        res[6 * n + 4] = sse;
        res[6 * n + 5] = svt_fast_loop_nxm_sad_kernel(pa, S, pb, S, (uint32_t)h, (uint32_t)w);
        int32_t *e = meta + 5 * n;
        e[0] = m, e[1] = oy, e[2] = ox, e[3] = w, e[4] = h;
    }
    golden_put2(&g, "meta", 'i', (uint32_t)N, 5, meta);
    golden_put2(&g, "res", 'I', (uint32_t)N, 6, res);
    golden_close(&g);
    free(A), free(B), free(A16), free(B16), free(meta), free(res);
}

/* ------------------------------------------------------------------------------------------- */
static void gen_cdef(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/cdef_shims.bin", dir);
    GoldenFile g = golden_open(path);
    Rng        r = {0x4344454600000001ull};
    /* 8xn: 12 x 12 windows (rows/cols -2..9) at stride 144, meta {bd, pri, sec, dir, pdamp, sdamp, ss}, 8 x 8 out */
    const int N    = 300;
    int32_t  *meta = calloc(N, 7 * sizeof(int32_t));
    uint16_t *win  = calloc(N, 12 * 12 * sizeof(uint16_t)), *out = calloc(N, 64 * sizeof(uint16_t));
    uint16_t  buf[144 * 12];
    for (int n = 0; n < N; n++) {
        const int bd = n % 3 == 0 ? 8 : n % 3 == 1 ? 10 : 12, cs = bd - 8, maxv = (1 << bd) - 1;
        const int ss = n % 5 == 0 ? 4 : n % 5 == 1 ? 2 : 1;
        const int pri = (int)rng_below(&r, 16) << cs, sec = ((int)rng_below(&r, 4) == 3 ? 4 : (int)rng_below(&r, 3)) << cs;
        const int d = (int)rng_below(&r, 8), damp = 3 + (int)rng_below(&r, 4) + cs;
        const int base = (int)rng_below(&r, (uint32_t)maxv + 1), amp = 1 + (int)rng_below(&r, (uint32_t)(maxv / 8 + 1));
        for (int k = 0; k < 144 * 12; k++) buf[k] = CDEF_VERY_LARGE;
        for (int y = 0; y < 12; y++)
            for (int x = 0; x < 12; x++) {
                uint16_t v = (uint16_t)clampi(base + (int)rng_below(&r, 2 * amp + 1) - amp, 0, maxv);
                if (rng_below(&r, 40) == 0) v = CDEF_VERY_LARGE; /* frame-edge padding samples */
                if (y >= 2 && y < 10 && x >= 2 && x < 10 && v == CDEF_VERY_LARGE) v = (uint16_t)base;
                buf[y * 144 + x] = v;
                win[(size_t)n * 144 + y * 12 + x] = v;
            }
        uint16_t *o = out + (size_t)n * 64;
        for (int k = 0; k < 64; k++) o[k] = 0xDEAD;
        svt_cdef_filter_block_8xn_16_avx2(buf + 2 * 144 + 2, pri, sec, d, damp, damp, cs, o, 8, 8, (uint8_t)ss);
        int32_t *m = meta + 7 * n;
        m[0] = bd, m[1] = pri, m[2] = sec, m[3] = d, m[4] = damp, m[5] = damp, m[6] = ss;
    }
    uint32_t d3[3] = {(uint32_t)N, 12, 12};
    golden_put(&g, "win", 'H', 3, d3, win);
    golden_put2(&g, "out", 'H', (uint32_t)N, 64, out);
    golden_put2(&g, "meta", 'i', (uint32_t)N, 7, meta);
    /* copy_rect8: 40 random rectangles out of a 70 x 90 8-bit buffer */
    uint8_t  src[70 * 90];
    uint16_t dst[40][70 * 90];
    int32_t  rm[40 * 2];
    for (int k = 0; k < 70 * 90; k++) src[k] = (uint8_t)rng_below(&r, 256);
    for (int n = 0; n < 40; n++) {
        const int v = 1 + (int)rng_below(&r, 70), h = 1 + (int)rng_below(&r, 90);
        for (int k = 0; k < 70 * 90; k++) dst[n][k] = 0xBEEF;
        svt_aom_copy_rect8_8bit_to_16bit_c(dst[n], 90, src, 90, v, h);
        rm[2 * n] = v, rm[2 * n + 1] = h;
    }
    golden_put2(&g, "rect_src", 'B', 70, 90, src);
    uint32_t d4[3] = {40, 70, 90};
    golden_put(&g, "rect_dst", 'H', 3, d4, dst);
    golden_put2(&g, "rect_meta", 'i', 40, 2, rm);
    golden_close(&g);
    free(meta), free(win), free(out);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    gen_proj(argv[1]);
    gen_md(argv[1]);
    gen_cdef(argv[1]);
    printf("shim golden vectors written to %s\n", argv[1]);
    return 0;
}
