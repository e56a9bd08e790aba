/*
 * frame_oracle.c — CPU restatement of the frame-buffer work around the path (TEST INFRASTRUCTURE: imported only by
 * tests/; never shipped or measured).  Pinned by tests/golden/frame_ops.bin (oracle/ref_harness/gen_golden_frame.c,
 * the reference's own C).
 *   oracle_convert    svt_convert_8bit_to_16bit_c / svt_convert_16bit_to_8bit_c (EbPackUnPack_C.c:270-283)
 *   oracle_pad        svt_aom_generate_padding / _16bit (EbMcp.c:95-150, 201-240): side borders of every visible row
 *                     from its edge samples, then the first / last padded row's whole stride over the top / bottom
 *   oracle_extend     svt_extend_frame (EbRestoration.c:160-203) around the visible area
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

void oracle_convert(const void *src, int sbits, int ss, void *dst, int dbits, int ds, int w, int h) {
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const unsigned v = sbits == 8 ? ((const uint8_t *)src)[(size_t)y * ss + x] : ((const uint16_t *)src)[(size_t)y * ss + x];
            if (dbits == 8) ((uint8_t *)dst)[(size_t)y * ds + x] = (uint8_t)v;
            else ((uint16_t *)dst)[(size_t)y * ds + x] = (uint16_t)v;
        }
}

#define DEF_PAD(T, name)                                                                                           \
    static void name(T *b, int stride, int w, int h, int pw, int ph) {                                              \
        for (int y = ph; y < ph + h; y++) {                                                                         \
            T *r = b + (size_t)y * stride;                                                                          \
            for (int i = 0; i < pw; i++) r[i] = r[pw], r[pw + w + i] = r[pw + w - 1];                               \
        }                                                                                                           \
        for (int y = 0; y < ph; y++) {                                                                              \
            memcpy(b + (size_t)y * stride, b + (size_t)ph * stride, sizeof(T) * stride);                            \
            memcpy(b + (size_t)(ph + h + y) * stride, b + (size_t)(ph + h - 1) * stride, sizeof(T) * stride);       \
        }                                                                                                           \
    }
DEF_PAD(uint8_t, pad8)
DEF_PAD(uint16_t, pad16)

void oracle_pad(void *buf, int bits, int stride, int w, int h, int pw, int ph) {
    if (bits == 8) pad8((uint8_t *)buf, stride, w, h, pw, ph);
    else pad16((uint16_t *)buf, stride, w, h, pw, ph);
}

#define DEF_EXT(T, name)                                                                                           \
    static void name(T *d, int stride, int w, int h, int bh, int bv) {                                              \
        for (int y = 0; y < h; y++) {                                                                               \
            T *r = d + (ptrdiff_t)y * stride;                                                                       \
            for (int i = 1; i <= bh; i++) r[-i] = r[0], r[w - 1 + i] = r[w - 1];                                    \
        }                                                                                                           \
        for (int y = 1; y <= bv; y++) {                                                                             \
            memcpy(d - (ptrdiff_t)y * stride - bh, d - bh, sizeof(T) * (w + 2 * bh));                               \
            memcpy(d + (ptrdiff_t)(h - 1 + y) * stride - bh, d + (ptrdiff_t)(h - 1) * stride - bh, sizeof(T) * (w + 2 * bh)); \
        }                                                                                                           \
    }
DEF_EXT(uint8_t, ext8)
DEF_EXT(uint16_t, ext16)

/* data = first visible sample */
void oracle_extend(void *data, int bits, int stride, int w, int h, int bh, int bv) {
    if (bits == 8) ext8((uint8_t *)data, stride, w, h, bh, bv);
    else ext16((uint16_t *)data, stride, w, h, bh, bv);
}
