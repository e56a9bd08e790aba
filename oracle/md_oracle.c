/*
 * md_oracle.c — CPU restatement of the mode-decision distortion kernels (SAD / SSE / variance).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Restates (paths under Source/Lib/):
 *   Encoder/C_DEFAULT/EbComputeSAD_C.c:39-56 (sad_16b_kernel), :92-206 (sad_inline_c, sad{W}x{H}, x4d)
 *   Encoder/C_DEFAULT/variance.c:256-345 (variance_c, VAR(W, H))
 *   Encoder/Codec/EbPsnr.c:146-214 (highbd_variance64, highbd_10_variance, HIGHBD_VAR(W, H))
 *   Encoder/Codec/EbEncInterPrediction.c:562-590 (svt_aom_sse_c, svt_aom_highbd_sse_c)
 *   Common/C_DEFAULT/EbPictureOperators_C.c:62-80, Common/Codec/EbPictureOperators.c:174-197
 * Pinned by tests/test_oracle_golden.py against tests/golden/md_*.bin (reference C outputs).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

uint32_t oracle_sad(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
    uint32_t s = 0;
    for (int y = 0; y < h; y++, a += as, b += bs)
        for (int x = 0; x < w; x++) s += (uint32_t)abs((int)a[x] - (int)b[x]);
    return s;
}

uint32_t oracle_sad16(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h) {
    uint32_t s = 0;
    for (int y = 0; y < h; y++, a += as, b += bs)
        for (int x = 0; x < w; x++) s += (uint32_t)abs((int)a[x] - (int)b[x]);
    return s;
}

/* svt_aom_variance{W}x{H}_c: 32-bit sse and sum, var = sse - sum^2 / (W*H) in uint32 */
uint32_t oracle_variance(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h, uint32_t *sse) {
    int      sum = 0;
    uint32_t s   = 0;
    for (int y = 0; y < h; y++, a += as, b += bs)
        for (int x = 0; x < w; x++) {
            const int d = (int)a[x] - (int)b[x];
            sum += d;
            s += (uint32_t)(d * d);
        }
    *sse = s;
    return s - (uint32_t)(((int64_t)sum * sum) / (w * h));
}

/* svt_aom_highbd_10_variance{W}x{H}_c: 64-bit accumulation, sse rounded >> 4, sum rounded >> 2,
 * var = max(0, sse - sum^2 / (W*H)) */
uint32_t oracle_highbd_10_variance(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h, uint32_t *sse) {
    int64_t  sum = 0;
    uint64_t s   = 0;
    for (int y = 0; y < h; y++, a += as, b += bs) {
        int32_t row = 0;
        for (int x = 0; x < w; x++) {
            const int d = (int)a[x] - (int)b[x];
            row += d;
            s += (uint32_t)(d * d);
        }
        sum += row;
    }
    *sse               = (uint32_t)((s + 8) >> 4);
    const int     rsum = (int)((sum + 2) >> 2);
    const int64_t var  = (int64_t)*sse - ((int64_t)rsum * rsum) / (w * h);
    return var >= 0 ? (uint32_t)var : 0;
}

int64_t oracle_sse(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
    int64_t s = 0;
    for (int y = 0; y < h; y++, a += as, b += bs)
        for (int x = 0; x < w; x++) s += ((int)a[x] - (int)b[x]) * ((int)a[x] - (int)b[x]);
    return s;
}

int64_t oracle_sse16(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h) {
    int64_t s = 0;
    for (int y = 0; y < h; y++, a += as, b += bs)
        for (int x = 0; x < w; x++) s += ((int)a[x] - (int)b[x]) * ((int)a[x] - (int)b[x]);
    return s;
}

/* ------------------------------------------------------------------------------------------- */
/* batch (the layout of svtgpu_md_dist_batch)                                                   */
/* ------------------------------------------------------------------------------------------- */
static const int kShapeW[19] = {4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 4, 16, 8, 32, 16, 64};
static const int kShapeH[19] = {4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 16, 4, 32, 8, 64, 16};

/* SBs [sb_begin, sb_end) only; out indexed from sb_begin (SB subsets of frames too large for the whole oracle) */
int oracle_md_dist_batch_range(const OracleFrame *src, const OracleFrame *const *refs, int nref, const int16_t *mv,
                               int sb_begin, int sb_end, uint32_t *out) {
    const int W = src->width, H = src->height, hb = src->bit_depth > 8;
    const int nsbx = (W + 63) / 64;
    uint16_t  s16[64 * 64], r16[64 * 64];
    uint8_t   s8[64 * 64], r8[64 * 64];
    for (int sb = sb_begin; sb < sb_end; sb++) {
        const int ox = (sb % nsbx) * 64, oy = (sb / nsbx) * 64;
        for (int y = 0; y < 64; y++)
            for (int x = 0; x < 64; x++) {
                const int cy = oy + y < H ? oy + y : H - 1, cx = ox + x < W ? ox + x : W - 1;
                const long i = (long)cy * src->stride[0] + cx;
                s16[y * 64 + x] = hb ? ((const uint16_t *)src->plane[0])[i] : ((const uint8_t *)src->plane[0])[i];
                s8[y * 64 + x]  = (uint8_t)s16[y * 64 + x];
            }
        for (int r = 0; r < nref; r++) {
            const OracleFrame *R  = refs[r];
            const int          mx = mv[((long)sb * nref + r) * 2], my = mv[((long)sb * nref + r) * 2 + 1];
            for (int y = 0; y < 64; y++)
                for (int x = 0; x < 64; x++) {
                    int cy = oy + y + my, cx = ox + x + mx;
                    cy            = cy < 0 ? 0 : cy >= H ? H - 1 : cy;
                    cx            = cx < 0 ? 0 : cx >= W ? W - 1 : cx;
                    const long i  = (long)cy * R->stride[0] + cx;
                    r16[y * 64 + x] = hb ? ((const uint16_t *)R->plane[0])[i] : ((const uint8_t *)R->plane[0])[i];
                    r8[y * 64 + x]  = (uint8_t)r16[y * 64 + x];
                }
            uint32_t *o = out + ((long)(sb - sb_begin) * nref + r) * 3 * SVTGPU_MD_BLOCKS;
            int       k = 0;
            for (int s = 0; s < 19; s++) {
                const int w = kShapeW[s], h = kShapeH[s];
                for (int by = 0; by < 64; by += h)
                    for (int bx = 0; bx < 64; bx += w, k++) {
                        const int off = by * 64 + bx;
                        uint32_t  sse, var;
                        if (hb) {
                            o[k] = oracle_sad16(s16 + off, 64, r16 + off, 64, w, h);
                            var  = oracle_highbd_10_variance(s16 + off, 64, r16 + off, 64, w, h, &sse);
                        } else {
                            o[k] = oracle_sad(s8 + off, 64, r8 + off, 64, w, h);
                            var  = oracle_variance(s8 + off, 64, r8 + off, 64, w, h, &sse);
                        }
                        o[SVTGPU_MD_BLOCKS + k]     = sse;
                        o[2 * SVTGPU_MD_BLOCKS + k] = var;
                    }
            }
        }
    }
    return SVTGPU_OK;
}

int oracle_md_dist_batch(const OracleFrame *src, const OracleFrame *const *refs, int nref, const int16_t *mv,
                         uint32_t *out) {
    return oracle_md_dist_batch_range(src, refs, nref, mv, 0, ((src->width + 63) / 64) * ((src->height + 63) / 64),
                                      out);
}
