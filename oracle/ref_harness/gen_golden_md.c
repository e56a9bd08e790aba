/*
 * gen_golden_md.c — mode-decision distortion golden vectors (test infrastructure; never shipped).
 *
 * Links the REFERENCE's own C kernels (EbComputeSAD_C.c, variance.c, EbPsnr.c, EbEncInterPrediction.c,
 * EbPictureOperators(_C).c, compiled from /root/reference by oracle/ref.mk) and records their outputs on
 * deterministic SplitMix64 blocks for all 22 AV1 block sizes, including the known-answer patterns of the
 * reference's tests (zero difference, maximum difference: VarianceTest.cc:346-387, HbdVarianceTest.cc:397-405).
 * usage: gen_golden_md <out_dir>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbDefinitions.h"
#include "aom_dsp_rtcd.h"
#include "common_dsp_rtcd.h"
#include "golden_io.h"

uint64_t svt_spatial_full_distortion_kernel_c(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                              uint8_t *recon, int32_t recon_offset, uint32_t recon_stride,
                                              uint32_t area_width, uint32_t area_height);
uint64_t svt_full_distortion_kernel16_bits_c(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                             uint8_t *pred, int32_t pred_offset, uint32_t pred_stride,
                                             uint32_t area_width, uint32_t area_height);

#define NSIZE 22
static const int kW[NSIZE] = {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 64, 128, 128, 4, 16, 8, 32, 16, 64};
static const int kH[NSIZE] = {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 128, 64, 128, 16, 4, 32, 8, 64, 16};
typedef uint32_t (*SadFn)(const uint8_t *, int, const uint8_t *, int);
typedef void (*Sad4dFn)(const uint8_t *, int, const uint8_t *const[], int, uint32_t *);
typedef unsigned int (*VarFn)(const uint8_t *, int, const uint8_t *, int, unsigned int *);
static const SadFn   kSad[NSIZE] = {
    svt_aom_sad4x4_c,
    svt_aom_sad4x8_c,
    svt_aom_sad8x4_c,
    svt_aom_sad8x8_c,
    svt_aom_sad8x16_c,
    svt_aom_sad16x8_c,
    svt_aom_sad16x16_c,
    svt_aom_sad16x32_c,
    svt_aom_sad32x16_c,
    svt_aom_sad32x32_c,
    svt_aom_sad32x64_c,
    svt_aom_sad64x32_c,
    svt_aom_sad64x64_c,
    svt_aom_sad64x128_c,
    svt_aom_sad128x64_c,
    svt_aom_sad128x128_c,
    svt_aom_sad4x16_c,
    svt_aom_sad16x4_c,
    svt_aom_sad8x32_c,
    svt_aom_sad32x8_c,
    svt_aom_sad16x64_c,
    svt_aom_sad64x16_c};
static const Sad4dFn kSad4d[NSIZE] = {
    svt_aom_sad4x4x4d_c,
    svt_aom_sad4x8x4d_c,
    svt_aom_sad8x4x4d_c,
    svt_aom_sad8x8x4d_c,
    svt_aom_sad8x16x4d_c,
    svt_aom_sad16x8x4d_c,
    svt_aom_sad16x16x4d_c,
    svt_aom_sad16x32x4d_c,
    svt_aom_sad32x16x4d_c,
    svt_aom_sad32x32x4d_c,
    svt_aom_sad32x64x4d_c,
    svt_aom_sad64x32x4d_c,
    svt_aom_sad64x64x4d_c,
    svt_aom_sad64x128x4d_c,
    svt_aom_sad128x64x4d_c,
    svt_aom_sad128x128x4d_c,
    svt_aom_sad4x16x4d_c,
    svt_aom_sad16x4x4d_c,
    svt_aom_sad8x32x4d_c,
    svt_aom_sad32x8x4d_c,
    svt_aom_sad16x64x4d_c,
    svt_aom_sad64x16x4d_c};
static const VarFn   kVar[NSIZE] = {
    svt_aom_variance4x4_c,
    svt_aom_variance4x8_c,
    svt_aom_variance8x4_c,
    svt_aom_variance8x8_c,
    svt_aom_variance8x16_c,
    svt_aom_variance16x8_c,
    svt_aom_variance16x16_c,
    svt_aom_variance16x32_c,
    svt_aom_variance32x16_c,
    svt_aom_variance32x32_c,
    svt_aom_variance32x64_c,
    svt_aom_variance64x32_c,
    svt_aom_variance64x64_c,
    svt_aom_variance64x128_c,
    svt_aom_variance128x64_c,
    svt_aom_variance128x128_c,
    svt_aom_variance4x16_c,
    svt_aom_variance16x4_c,
    svt_aom_variance8x32_c,
    svt_aom_variance32x8_c,
    svt_aom_variance16x64_c,
    svt_aom_variance64x16_c};
static const VarFn   kHVar[NSIZE] = {
    svt_aom_highbd_10_variance4x4_c,
    svt_aom_highbd_10_variance4x8_c,
    svt_aom_highbd_10_variance8x4_c,
    svt_aom_highbd_10_variance8x8_c,
    svt_aom_highbd_10_variance8x16_c,
    svt_aom_highbd_10_variance16x8_c,
    svt_aom_highbd_10_variance16x16_c,
    svt_aom_highbd_10_variance16x32_c,
    svt_aom_highbd_10_variance32x16_c,
    svt_aom_highbd_10_variance32x32_c,
    svt_aom_highbd_10_variance32x64_c,
    svt_aom_highbd_10_variance64x32_c,
    svt_aom_highbd_10_variance64x64_c,
    svt_aom_highbd_10_variance64x128_c,
    svt_aom_highbd_10_variance128x64_c,
    svt_aom_highbd_10_variance128x128_c,
    svt_aom_highbd_10_variance4x16_c,
    svt_aom_highbd_10_variance16x4_c,
    svt_aom_highbd_10_variance8x32_c,
    svt_aom_highbd_10_variance32x8_c,
    svt_aom_highbd_10_variance16x64_c,
    svt_aom_highbd_10_variance64x16_c};

#define NCASE 6 /* per size: 0 = zero diff, 1 = max diff, 2.. = random (smooth + noise, full range) */
static int STRIDE; /* per size: w + 8 (a stride wider than the block; x4d reads 2 columns further) */

static void fill(Rng *r, uint16_t *src, uint16_t *ref, int w, int h, int kind) {
    const int base = (int)rng_below(r, 1024);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < STRIDE; x++) {
            int s, d;
            if (kind == 0) {
                s = (int)rng_below(r, 1024);
                d = s;
            } else if (kind == 1) {
                s = 1023;
                d = 0;
            } else if (kind == 2 || kind == 3) {
                s = (int)rng_below(r, 1024);
                d = (int)rng_below(r, 1024);
            } else {
                s = base + (x + y) / 2 + (int)rng_below(r, 9) - 4;
                d = s + (int)rng_below(r, 41) - 20;
            }
            src[y * STRIDE + x] = (uint16_t)(s < 0 ? 0 : s > 1023 ? 1023 : s);
            ref[y * STRIDE + x] = (uint16_t)(d < 0 ? 0 : d > 1023 ? 1023 : d);
        }
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    char path[512];
    snprintf(path, sizeof path, "%s/md_dist.bin", argv[1]);
    GoldenFile g = golden_open(path);
    Rng        r = {0x3D00000000000001ull};
    for (int si = 0; si < NSIZE; si++) {
        const int w = kW[si], h = kH[si];
        STRIDE      = w + 8;
        /* inputs: 10-bit samples (the 8-bit kernels see the low 8 bits) */
        uint16_t *src = malloc(sizeof(uint16_t) * STRIDE * (h + 3) * NCASE);
        uint16_t *ref = malloc(sizeof(uint16_t) * STRIDE * (h + 3) * NCASE);
        uint32_t  res[NCASE][12];
        for (int c = 0; c < NCASE; c++) {
            uint16_t *s = src + (size_t)c * STRIDE * (h + 3), *d = ref + (size_t)c * STRIDE * (h + 3);
            fill(&r, s, d, w, h + 3, c);
            uint8_t *s8 = malloc((size_t)STRIDE * (h + 3)), *d8 = malloc((size_t)STRIDE * (h + 3));
            for (int k = 0; k < STRIDE * (h + 3); k++) s8[k] = c == 1 ? 255 : (uint8_t)s[k];
            for (int k = 0; k < STRIDE * (h + 3); k++) d8[k] = c == 1 ? 0 : (uint8_t)d[k];
            unsigned int sse = 0;
            res[c][0] = kSad[si](s8, STRIDE, d8, STRIDE);
            res[c][1] = kVar[si](s8, STRIDE, d8, STRIDE, &sse);
            res[c][2] = sse;
            res[c][3] = kHVar[si](CONVERT_TO_BYTEPTR(s), STRIDE, CONVERT_TO_BYTEPTR(d), STRIDE, &sse);
            res[c][4] = sse;
            res[c][5] = svt_aom_sad_16b_kernel_c(s, STRIDE, d, STRIDE, h, w);
            const uint8_t *refs4[4] = {d8, d8 + 1, d8 + STRIDE, d8 + 3 * STRIDE + 2};
            uint32_t       s4[4];
            kSad4d[si](s8, STRIDE, refs4, STRIDE, s4);
            memcpy(&res[c][6], s4, sizeof s4);
            const int64_t e8  = svt_aom_sse_c(s8, STRIDE, d8, STRIDE, w, h);
            const int64_t e16 = svt_aom_highbd_sse_c((const uint8_t *)s, STRIDE, (const uint8_t *)d, STRIDE, w, h);
            const uint64_t f8 = svt_spatial_full_distortion_kernel_c(s8, 0, STRIDE, d8, 0, STRIDE, w, h);
            const uint64_t f16 = svt_full_distortion_kernel16_bits_c((uint8_t *)s, 0, STRIDE, (uint8_t *)d, 0, STRIDE, w, h);
            if ((uint64_t)e8 != f8 || (uint64_t)e16 != f16) {
                fprintf(stderr, "sse mismatch between reference kernels\n");
                return 1;
            }
            res[c][10] = (uint32_t)e8;  /* < 2^32 for every size at 8 bit */
            res[c][11] = (uint32_t)(e16 >> 4);
            free(s8);
            free(d8);
        }
        char nm[64];
        uint32_t dims[3] = {NCASE, (uint32_t)(h + 3), STRIDE};
        snprintf(nm, sizeof nm, "s%d_src", si);
        golden_put(&g, nm, 'H', 3, dims, src);
        snprintf(nm, sizeof nm, "s%d_ref", si);
        golden_put(&g, nm, 'H', 3, dims, ref);
        snprintf(nm, sizeof nm, "s%d_res", si);
        golden_put2(&g, nm, 'I', NCASE, 12, res);
        free(src);
        free(ref);
    }
    golden_close(&g);
    printf("md golden vectors written to %s\n", argv[1]);
    return 0;
}
