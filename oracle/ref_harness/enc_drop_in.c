/*
 * enc_drop_in.c — libsvtgpu inside the reference encoder (test infrastructure, never shipped).
 *
 * Drives the reference's own encoder library (oracle/enc.mk: every C source of Source/Lib/{Common,Encoder} compiled
 * C-only into oracle/_ref/enc/libsvtenc.so) through its public API -- svt_av1_enc_init_handle / _set_parameter /
 * _init / _send_picture / _get_packet (Source/API/EbSvtAv1Enc.h:989-1079) -- over a synthetic 10-bit 4:2:0 clip with
 * deblocking, CDEF and loop restoration (Wiener + self-guided) on, and writes the bitstream.  Modes:
 *   cpu    the reference encoder as built (its C kernels);
 *   rtcd   the same, with include/svtgpu_rtcd.h's svtgpu_install_filter_rtcd() called right after svt_av1_enc_init:
 *          the encoder's DLF / CDEF / LR / full-distortion RTCD pointers (read at call time by svt_aom_dlf_kernel,
 *          svt_aom_cdef_kernel, svt_aom_rest_kernel and mode decision) now run libsvtgpu's device kernels;
 *   frame  the frame-level entry points alone (the RTCD pointers stay the encoder's C): enc_frame_hooks.c defines the encoder's frame-level filter calls
 *          (svt_av1_pick_filter_level, svt_av1_loop_filter_frame, finish_cdef_search, svt_av1_cdef_frame,
 *          rest_finish_search, svt_av1_loop_restoration_filter_frame; EbDlfProcess.c:55-153, EbCdefProcess.c:364-738,
 *          EbRestProcess.c:520-640) in this executable; ELF symbol interposition makes the library's calls land on them,
 *          so the reference sources are compiled unmodified and the process bodies call libsvtgpu's frame-level API.
 * tests/test_encoder_drop_in.py compares the three bitstreams byte for byte.
 *
 *   enc_drop_in <cpu|rtcd|frame> <out.obu> [width height frames preset qp bit_depth logical_processors]
 * (bit_depth 8 or 10, default 10: an 8-bit clip runs the encoder's 8-bit pipeline; logical_processors > 1: several
 * pictures through the encoder's DLF / CDEF / REST processes at once)
 * Prints one line: "<mode> bytes <n> packets <n> shim_calls <n> frame_calls <n> frame_fallbacks <n>".
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "EbSvtAv1Enc.h"
#include "EbDefinitions.h"
#include "aom_dsp_rtcd.h"
#include "common_dsp_rtcd.h"
#include "EbMcp.h"
#include "svtgpu_rtcd.h"

uint64_t enc_frame_hook_calls(void); /* enc_frame_hooks.c: hooked frame-level calls served by libsvtgpu */
uint64_t enc_frame_hook_fallbacks(void); /* ... and those left to the encoder's own function */
void     enc_frame_hooks_enable(int on);
void     enc_frame_hook_kinds(uint64_t out[10]);

/* a deterministic synthetic 10-bit picture: gradients, a moving disc, texture and noise (LCG) */
static void fill_frame(uint16_t *y, uint16_t *u, uint16_t *v, int w, int h, int k) {
    uint32_t s = 0x5EED0000u + 7919u * (uint32_t)k;
    const int cx = w / 3 + 6 * k, cy = h / 2 + 3 * k, r = h / 5;
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            s         = s * 1664525u + 1013904223u;
            int val   = 200 + (j * 400) / w + (i * 200) / h + (int)((s >> 24) & 15) - 8;
            const int dx = j - cx, dy = i - cy;
            if (dx * dx + dy * dy < r * r) val += 250;
            if (((i / 8) + (j / 8) + k) % 7 == 0) val += ((i ^ j) & 31) * 3;
            y[i * w + j] = (uint16_t)(val < 0 ? 0 : val > 1023 ? 1023 : val);
        }
    for (int i = 0; i < h / 2; i++)
        for (int j = 0; j < w / 2; j++) {
            s                      = s * 1664525u + 1013904223u;
            u[i * (w / 2) + j] = (uint16_t)(480 + (j * 60) / w + (int)((s >> 25) & 7));
            v[i * (w / 2) + j] = (uint16_t)(560 - (i * 80) / h + (int)((s >> 26) & 3) + ((j + k) % 13 == 0 ? 20 : 0));
        }
}

static int check(EbErrorType e, const char *what) {
    if (e != EB_ErrorNone) {
        fprintf(stderr, "enc_drop_in: %s failed: 0x%x\n", what, (unsigned)e);
        exit(2);
    }
    return 0;
}

static int in_libsvtgpu(const void *f) {
    Dl_info d;
    return f && dladdr(f, &d) && d.dli_fname && strstr(d.dli_fname, "libsvtgpu") != NULL;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: enc_drop_in <cpu|rtcd|frame> <out.obu> [width height frames preset qp bit_depth lp]\n");
        return 2;
    }
    const char *mode   = argv[1];
    const int   rtcd   = !strcmp(mode, "rtcd");
    const int   frame  = !strcmp(mode, "frame");
    const int   w      = argc > 3 ? atoi(argv[3]) : 320;
    const int   h      = argc > 4 ? atoi(argv[4]) : 192;
    const int   nfr    = argc > 5 ? atoi(argv[5]) : 5;
    const int   preset = argc > 6 ? atoi(argv[6]) : 2;
    const int   qp     = argc > 7 ? atoi(argv[7]) : 40;
    const int   bd     = argc > 8 ? atoi(argv[8]) : 10;
    const int   lp     = argc > 9 ? atoi(argv[9]) : 1;
    if (bd != 8 && bd != 10) return 2;
    if (!rtcd && !frame && strcmp(mode, "cpu")) return 2;
    if ((rtcd || frame) && !svtgpu_device_available()) {
        fprintf(stderr, "enc_drop_in: no gfx950 device\n");
        return 3;
    }
    FILE *out = fopen(argv[2], "wb");
    if (!out) return 2;

    EbComponentType         *enc = NULL;
    EbSvtAv1EncConfiguration cfg;
    check(svt_av1_enc_init_handle(&enc, NULL, &cfg), "svt_av1_enc_init_handle");
    cfg.enc_mode                     = (int8_t)preset;
    cfg.source_width                 = (uint32_t)w;
    cfg.source_height                = (uint32_t)h;
    cfg.encoder_bit_depth            = (uint32_t)bd;
    cfg.encoder_color_format         = EB_YUV420;
    cfg.frame_rate_numerator         = 30;
    cfg.frame_rate_denominator       = 1;
    cfg.rate_control_mode            = 0; /* CQP */
    cfg.enable_adaptive_quantization = 0;
    cfg.qp                           = (uint32_t)qp;
    cfg.intra_period_length          = -1;
    cfg.enable_dlf_flag              = TRUE;
    cfg.cdef_level                   = DEFAULT;
    cfg.enable_restoration_filtering = 1;
    cfg.logical_processors           = (uint32_t)lp;
    check(svt_av1_enc_set_parameter(enc, &cfg), "svt_av1_enc_set_parameter");
    check(svt_av1_enc_init(enc), "svt_av1_enc_init");
    /* the RTCD setup ran inside svt_av1_enc_init (EbEncHandle.c:1530-1531); no picture has been sent yet, and the
       filter pointers are read at call time: install here */
    int installed = 0;
    if (rtcd) {
        svtgpu_install_filter_rtcd();
        const void *p[] = {(const void *)svt_cdef_filter_block, (const void *)svt_aom_highbd_lpf_vertical_14,
                           (const void *)svt_av1_selfguided_restoration, (const void *)svt_av1_compute_stats_highbd,
                           (const void *)svt_full_distortion_kernel16_bits};
        for (int i = 0; i < 5; i++) installed += in_libsvtgpu(p[i]);
        if (installed != 5) {
            fprintf(stderr, "enc_drop_in: install failed (%d/5 pointers in libsvtgpu)\n", installed);
            return 4;
        }
    }
    enc_frame_hooks_enable(frame);

    EbBufferHeaderType *hdr = NULL;
    check(svt_av1_enc_stream_header(enc, &hdr), "svt_av1_enc_stream_header");
    fwrite(hdr->p_buffer, 1, hdr->n_filled_len, out);
    size_t total = hdr->n_filled_len;
    svt_av1_enc_stream_header_release(hdr);

    uint16_t *y = malloc((size_t)w * h * 2), *u = malloc((size_t)w * h / 2), *v = malloc((size_t)w * h / 2);
    /* the 8-bit clip: the same pictures >> 2 */
    uint8_t *y8 = malloc((size_t)w * h), *u8 = malloc((size_t)w * h / 4), *v8 = malloc((size_t)w * h / 4);
    int       got = 0, done = 0;
    for (int k = 0; k <= nfr && !done; k++) {
        EbBufferHeaderType in;
        EbSvtIOFormat      pic;
        memset(&in, 0, sizeof in);
        memset(&pic, 0, sizeof pic);
        in.size = sizeof in;
        if (k < nfr) {
            fill_frame(y, u, v, w, h, k);
            if (bd == 8) {
                for (size_t i = 0; i < (size_t)w * h; i++) y8[i] = (uint8_t)(y[i] >> 2);
                for (size_t i = 0; i < (size_t)w * h / 4; i++) u8[i] = (uint8_t)(u[i] >> 2), v8[i] = (uint8_t)(v[i] >> 2);
                pic.luma = y8, pic.cb = u8, pic.cr = v8;
            } else {
                pic.luma = (uint8_t *)y, pic.cb = (uint8_t *)u, pic.cr = (uint8_t *)v;
            }
            pic.y_stride = (uint32_t)w, pic.cb_stride = pic.cr_stride = (uint32_t)(w / 2);
            pic.width = (uint32_t)w, pic.height = (uint32_t)h;
            pic.color_fmt = EB_YUV420, pic.bit_depth = bd == 8 ? EB_EIGHT_BIT : EB_TEN_BIT;
            in.p_buffer     = (uint8_t *)&pic;
            in.n_filled_len = (uint32_t)((size_t)w * h * 3 / (bd == 8 ? 2 : 1));
            in.n_alloc_len  = in.n_filled_len;
            in.pts          = k;
            in.pic_type     = EB_AV1_INVALID_PICTURE;
        } else
            in.flags = EB_BUFFERFLAG_EOS;
        check(svt_av1_enc_send_picture(enc, &in), "svt_av1_enc_send_picture");
        /* drain what is ready; after the EOS picture, block until the EOS packet */
        for (;;) {
            EbBufferHeaderType *pkt = NULL;
            EbErrorType         e   = svt_av1_enc_get_packet(enc, &pkt, k == nfr);
            if (e == EB_NoErrorEmptyQueue) break;
            check(e, "svt_av1_enc_get_packet");
            fwrite(pkt->p_buffer, 1, pkt->n_filled_len, out);
            total += pkt->n_filled_len;
            got++;
            const int eos = (pkt->flags & EB_BUFFERFLAG_EOS) != 0;
            svt_av1_enc_release_out_buffer(&pkt);
            if (eos) {
                done = 1;
                break;
            }
        }
    }
    fclose(out);
    check(svt_av1_enc_deinit(enc), "svt_av1_enc_deinit");
    check(svt_av1_enc_deinit_handle(enc), "svt_av1_enc_deinit_handle");
    printf("%s bytes %zu packets %d shim_calls %llu frame_calls %llu frame_fallbacks %llu\n", mode, total, got,
           (unsigned long long)(rtcd || frame ? svtgpu_shim_calls() : 0), (unsigned long long)enc_frame_hook_calls(),
           (unsigned long long)enc_frame_hook_fallbacks());
    if (frame) {
        uint64_t k[10];
        enc_frame_hook_kinds(k);
        printf("frame kinds dlf_pick %llu dlf_frame %llu cdef_pick %llu cdef_apply %llu lr_search %llu lr_apply %llu "
               "lr_on %llu ccso_search %llu ccso_apply %llu ccso_on %llu\n", (unsigned long long)k[0],
               (unsigned long long)k[1], (unsigned long long)k[2], (unsigned long long)k[3], (unsigned long long)k[4],
               (unsigned long long)k[5], (unsigned long long)k[6], (unsigned long long)k[7], (unsigned long long)k[8],
               (unsigned long long)k[9]);
    }
    free(y), free(u), free(v), free(y8), free(u8), free(v8);
    return 0;
}
