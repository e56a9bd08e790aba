/*
 * svtgpu_rtcd.h — installs libsvtgpu's per-block shims into the SVT-AV1 encoder's RTCD function pointers.
 *
 * Include it in ONE translation unit of the encoder that sees the reference's RTCD declarations (common_dsp_rtcd.h,
 * aom_dsp_rtcd.h, EbMcp.h) and call the install functions between the RTCD setup and the first copy of those pointers:
 *
 *     svt_aom_setup_common_rtcd_internal(...);            // EbEncHandle.c:1530
 *     svt_aom_setup_rtcd_internal(...);                   // EbEncHandle.c:1531 (SET_FUNCTIONS may set a pointer once,
 *                                                         //   aom_dsp_rtcd.c:56-68, so install after it)
 *     if (getenv("SVT_GPU") && svtgpu_device_available()) {
 *         svtgpu_install_filter_rtcd();                   // the in-loop filter path (DLF / CDEF / LR)
 *         svtgpu_install_me_md_rtcd();                    // ME / MD distortion + frame buffers
 *         svtgpu_install_ccso_rtcd();                     // CCSO's block kernels (an encoder that re-enables it)
 *     }
 *     ...
 *     init_fn_ptr();                                      // EbEncHandle.c:1546: av1me.c:31 COPIES the sad / variance /
 *                                                         //   sub-pixel variance / x4d pointers into svt_aom_mefn_ptr[],
 *                                                         //   which MD and ME call (EbProductCodingLoop.c:999, ...);
 *                                                         //   an install after this line leaves those calls on the CPU
 *
 * (tests/test_rtcd_bind.py: oracle/_ref/rtcd_install runs this order against the reference's own init_fn_ptr and
 * checks every svt_aom_mefn_ptr[] entry, and the opposite order.)
 *
 * Every shim prototype names the reference's own types through the type hooks of svtgpu.h, so each assignment below
 * compiles under -Werror=incompatible-pointer-types without a cast.  The shims are synchronous per-block entry points
 * (the reference's unit tests run against the device through them); the fast path is the frame-level API.
 */
#ifndef SVTGPU_RTCD_H
#define SVTGPU_RTCD_H
#ifndef SVTGPU_CDEF_LIST_T
#define SVTGPU_CDEF_LIST_T CdefList
#endif
#ifndef SVTGPU_BLOCK_SIZE_T
#define SVTGPU_BLOCK_SIZE_T BlockSize
#endif
#ifndef SVTGPU_SGR_PARAMS_T
#define SVTGPU_SGR_PARAMS_T SgrParamsType
#endif
#ifndef SVTGPU_CONVOLVE_PARAMS_T
#define SVTGPU_CONVOLVE_PARAMS_T ConvolveParams
#endif
#ifndef SVTGPU_BIT_DEPTH_T
#define SVTGPU_BIT_DEPTH_T EbBitDepth
#endif
#include "svtgpu.h"

/* the in-loop filter path: loop filter x16, CDEF, Wiener / self-guided filters and statistics, the full-distortion
 * kernels (common_dsp_rtcd.h, aom_dsp_rtcd.h) */
static inline void svtgpu_install_filter_rtcd(void) {
    svt_aom_lpf_horizontal_4               = svtgpu_lpf_horizontal_4;
    svt_aom_lpf_horizontal_6               = svtgpu_lpf_horizontal_6;
    svt_aom_lpf_horizontal_8               = svtgpu_lpf_horizontal_8;
    svt_aom_lpf_horizontal_14              = svtgpu_lpf_horizontal_14;
    svt_aom_lpf_vertical_4                 = svtgpu_lpf_vertical_4;
    svt_aom_lpf_vertical_6                 = svtgpu_lpf_vertical_6;
    svt_aom_lpf_vertical_8                 = svtgpu_lpf_vertical_8;
    svt_aom_lpf_vertical_14                = svtgpu_lpf_vertical_14;
    svt_aom_highbd_lpf_horizontal_4        = svtgpu_highbd_lpf_horizontal_4;
    svt_aom_highbd_lpf_horizontal_6        = svtgpu_highbd_lpf_horizontal_6;
    svt_aom_highbd_lpf_horizontal_8        = svtgpu_highbd_lpf_horizontal_8;
    svt_aom_highbd_lpf_horizontal_14       = svtgpu_highbd_lpf_horizontal_14;
    svt_aom_highbd_lpf_vertical_4          = svtgpu_highbd_lpf_vertical_4;
    svt_aom_highbd_lpf_vertical_6          = svtgpu_highbd_lpf_vertical_6;
    svt_aom_highbd_lpf_vertical_8          = svtgpu_highbd_lpf_vertical_8;
    svt_aom_highbd_lpf_vertical_14         = svtgpu_highbd_lpf_vertical_14;
    svt_spatial_full_distortion_kernel     = svtgpu_spatial_full_distortion_kernel;
    svt_full_distortion_kernel16_bits      = svtgpu_full_distortion_kernel16_bits;
    svt_cdef_filter_block                  = svtgpu_cdef_filter_block;
    svt_cdef_filter_block_8xn_16           = svtgpu_cdef_filter_block_8xn_16;
    svt_aom_cdef_find_dir                  = svtgpu_cdef_find_dir;
    svt_aom_cdef_find_dir_dual             = svtgpu_cdef_find_dir_dual;
    svt_compute_cdef_dist_16bit            = svtgpu_compute_cdef_dist_16bit;
    svt_compute_cdef_dist_8bit             = svtgpu_compute_cdef_dist_8bit;
    svt_search_one_dual                    = svtgpu_search_one_dual;
    svt_aom_copy_rect8_8bit_to_16bit       = svtgpu_aom_copy_rect8_8bit_to_16bit;
    svt_av1_wiener_convolve_add_src        = svtgpu_av1_wiener_convolve_add_src;
    svt_av1_highbd_wiener_convolve_add_src = svtgpu_av1_highbd_wiener_convolve_add_src;
    svt_av1_selfguided_restoration         = svtgpu_av1_selfguided_restoration;
    svt_apply_selfguided_restoration       = svtgpu_apply_selfguided_restoration;
    svt_av1_compute_stats                  = svtgpu_av1_compute_stats;
    svt_av1_compute_stats_highbd           = svtgpu_av1_compute_stats_highbd;
    svt_get_proj_subspace                  = svtgpu_get_proj_subspace;
    svt_av1_lowbd_pixel_proj_error         = svtgpu_av1_lowbd_pixel_proj_error;
    svt_av1_highbd_pixel_proj_error        = svtgpu_av1_highbd_pixel_proj_error;
    svt_aom_mse16x16                       = svtgpu_aom_mse16x16;
    svt_aom_highbd_8_mse16x16              = svtgpu_aom_highbd_8_mse16x16;
}

/* CCSO's per-block kernels (common_dsp_rtcd.h:1025-1090), for an encoder that re-enables the fork's CCSO search /
 * apply (EbCdefProcess.c:621-623); the frame-level path is svtgpu_ccso_search_frame + svtgpu_ccso_apply_plane */
static inline void svtgpu_install_ccso_rtcd(void) {
    ccso_filter_block_hbd_wo_buf   = svtgpu_ccso_filter_block_hbd_wo_buf;
    ccso_filter_block_hbd_with_buf = svtgpu_ccso_filter_block_hbd_with_buf;
    ccso_derive_src_block          = svtgpu_ccso_derive_src_block;
    compute_distortion_block       = svtgpu_compute_distortion_block;
}

/* ME and MD distortion (every SAD / x4d / variance / highbd variance / sub-pixel variance size, sse, the open-loop ME
 * and MD full-pel search kernels) and the 8 <-> 16-bit frame conversions (aom_dsp_rtcd.h, common_dsp_rtcd.h) */
static inline void svtgpu_install_me_md_rtcd(void) {
    svt_aom_highbd_10_variance128x128         = svtgpu_aom_highbd_10_variance128x128;
    svt_aom_highbd_10_variance128x64          = svtgpu_aom_highbd_10_variance128x64;
    svt_aom_highbd_10_variance16x16           = svtgpu_aom_highbd_10_variance16x16;
    svt_aom_highbd_10_variance16x32           = svtgpu_aom_highbd_10_variance16x32;
    svt_aom_highbd_10_variance16x4            = svtgpu_aom_highbd_10_variance16x4;
    svt_aom_highbd_10_variance16x64           = svtgpu_aom_highbd_10_variance16x64;
    svt_aom_highbd_10_variance16x8            = svtgpu_aom_highbd_10_variance16x8;
    svt_aom_highbd_10_variance32x16           = svtgpu_aom_highbd_10_variance32x16;
    svt_aom_highbd_10_variance32x32           = svtgpu_aom_highbd_10_variance32x32;
    svt_aom_highbd_10_variance32x64           = svtgpu_aom_highbd_10_variance32x64;
    svt_aom_highbd_10_variance32x8            = svtgpu_aom_highbd_10_variance32x8;
    svt_aom_highbd_10_variance4x16            = svtgpu_aom_highbd_10_variance4x16;
    svt_aom_highbd_10_variance4x4             = svtgpu_aom_highbd_10_variance4x4;
    svt_aom_highbd_10_variance4x8             = svtgpu_aom_highbd_10_variance4x8;
    svt_aom_highbd_10_variance64x128          = svtgpu_aom_highbd_10_variance64x128;
    svt_aom_highbd_10_variance64x16           = svtgpu_aom_highbd_10_variance64x16;
    svt_aom_highbd_10_variance64x32           = svtgpu_aom_highbd_10_variance64x32;
    svt_aom_highbd_10_variance64x64           = svtgpu_aom_highbd_10_variance64x64;
    svt_aom_highbd_10_variance8x16            = svtgpu_aom_highbd_10_variance8x16;
    svt_aom_highbd_10_variance8x32            = svtgpu_aom_highbd_10_variance8x32;
    svt_aom_highbd_10_variance8x4             = svtgpu_aom_highbd_10_variance8x4;
    svt_aom_highbd_10_variance8x8             = svtgpu_aom_highbd_10_variance8x8;
    svt_aom_highbd_sse                        = svtgpu_aom_highbd_sse;
    svt_aom_sad128x128                        = svtgpu_aom_sad128x128;
    svt_aom_sad128x128x4d                     = svtgpu_aom_sad128x128x4d;
    svt_aom_sad128x64                         = svtgpu_aom_sad128x64;
    svt_aom_sad128x64x4d                      = svtgpu_aom_sad128x64x4d;
    svt_aom_sad16x16                          = svtgpu_aom_sad16x16;
    svt_aom_sad16x16x4d                       = svtgpu_aom_sad16x16x4d;
    svt_aom_sad16x32                          = svtgpu_aom_sad16x32;
    svt_aom_sad16x32x4d                       = svtgpu_aom_sad16x32x4d;
    svt_aom_sad16x4                           = svtgpu_aom_sad16x4;
    svt_aom_sad16x4x4d                        = svtgpu_aom_sad16x4x4d;
    svt_aom_sad16x64                          = svtgpu_aom_sad16x64;
    svt_aom_sad16x64x4d                       = svtgpu_aom_sad16x64x4d;
    svt_aom_sad16x8                           = svtgpu_aom_sad16x8;
    svt_aom_sad16x8x4d                        = svtgpu_aom_sad16x8x4d;
    svt_aom_sad32x16                          = svtgpu_aom_sad32x16;
    svt_aom_sad32x16x4d                       = svtgpu_aom_sad32x16x4d;
    svt_aom_sad32x32                          = svtgpu_aom_sad32x32;
    svt_aom_sad32x32x4d                       = svtgpu_aom_sad32x32x4d;
    svt_aom_sad32x64                          = svtgpu_aom_sad32x64;
    svt_aom_sad32x64x4d                       = svtgpu_aom_sad32x64x4d;
    svt_aom_sad32x8                           = svtgpu_aom_sad32x8;
    svt_aom_sad32x8x4d                        = svtgpu_aom_sad32x8x4d;
    svt_aom_sad4x16                           = svtgpu_aom_sad4x16;
    svt_aom_sad4x16x4d                        = svtgpu_aom_sad4x16x4d;
    svt_aom_sad4x4                            = svtgpu_aom_sad4x4;
    svt_aom_sad4x4x4d                         = svtgpu_aom_sad4x4x4d;
    svt_aom_sad4x8                            = svtgpu_aom_sad4x8;
    svt_aom_sad4x8x4d                         = svtgpu_aom_sad4x8x4d;
    svt_aom_sad64x128                         = svtgpu_aom_sad64x128;
    svt_aom_sad64x128x4d                      = svtgpu_aom_sad64x128x4d;
    svt_aom_sad64x16                          = svtgpu_aom_sad64x16;
    svt_aom_sad64x16x4d                       = svtgpu_aom_sad64x16x4d;
    svt_aom_sad64x32                          = svtgpu_aom_sad64x32;
    svt_aom_sad64x32x4d                       = svtgpu_aom_sad64x32x4d;
    svt_aom_sad64x64                          = svtgpu_aom_sad64x64;
    svt_aom_sad64x64x4d                       = svtgpu_aom_sad64x64x4d;
    svt_aom_sad8x16                           = svtgpu_aom_sad8x16;
    svt_aom_sad8x16x4d                        = svtgpu_aom_sad8x16x4d;
    svt_aom_sad8x32                           = svtgpu_aom_sad8x32;
    svt_aom_sad8x32x4d                        = svtgpu_aom_sad8x32x4d;
    svt_aom_sad8x4                            = svtgpu_aom_sad8x4;
    svt_aom_sad8x4x4d                         = svtgpu_aom_sad8x4x4d;
    svt_aom_sad8x8                            = svtgpu_aom_sad8x8;
    svt_aom_sad8x8x4d                         = svtgpu_aom_sad8x8x4d;
    svt_aom_sse                               = svtgpu_aom_sse;
    svt_aom_sub_pixel_variance128x128         = svtgpu_aom_sub_pixel_variance128x128;
    svt_aom_sub_pixel_variance128x64          = svtgpu_aom_sub_pixel_variance128x64;
    svt_aom_sub_pixel_variance16x16           = svtgpu_aom_sub_pixel_variance16x16;
    svt_aom_sub_pixel_variance16x32           = svtgpu_aom_sub_pixel_variance16x32;
    svt_aom_sub_pixel_variance16x4            = svtgpu_aom_sub_pixel_variance16x4;
    svt_aom_sub_pixel_variance16x64           = svtgpu_aom_sub_pixel_variance16x64;
    svt_aom_sub_pixel_variance16x8            = svtgpu_aom_sub_pixel_variance16x8;
    svt_aom_sub_pixel_variance32x16           = svtgpu_aom_sub_pixel_variance32x16;
    svt_aom_sub_pixel_variance32x32           = svtgpu_aom_sub_pixel_variance32x32;
    svt_aom_sub_pixel_variance32x64           = svtgpu_aom_sub_pixel_variance32x64;
    svt_aom_sub_pixel_variance32x8            = svtgpu_aom_sub_pixel_variance32x8;
    svt_aom_sub_pixel_variance4x16            = svtgpu_aom_sub_pixel_variance4x16;
    svt_aom_sub_pixel_variance4x4             = svtgpu_aom_sub_pixel_variance4x4;
    svt_aom_sub_pixel_variance4x8             = svtgpu_aom_sub_pixel_variance4x8;
    svt_aom_sub_pixel_variance64x128          = svtgpu_aom_sub_pixel_variance64x128;
    svt_aom_sub_pixel_variance64x16           = svtgpu_aom_sub_pixel_variance64x16;
    svt_aom_sub_pixel_variance64x32           = svtgpu_aom_sub_pixel_variance64x32;
    svt_aom_sub_pixel_variance64x64           = svtgpu_aom_sub_pixel_variance64x64;
    svt_aom_sub_pixel_variance8x16            = svtgpu_aom_sub_pixel_variance8x16;
    svt_aom_sub_pixel_variance8x32            = svtgpu_aom_sub_pixel_variance8x32;
    svt_aom_sub_pixel_variance8x4             = svtgpu_aom_sub_pixel_variance8x4;
    svt_aom_sub_pixel_variance8x8             = svtgpu_aom_sub_pixel_variance8x8;
    svt_aom_variance128x128                   = svtgpu_aom_variance128x128;
    svt_aom_variance128x64                    = svtgpu_aom_variance128x64;
    svt_aom_variance16x16                     = svtgpu_aom_variance16x16;
    svt_aom_variance16x32                     = svtgpu_aom_variance16x32;
    svt_aom_variance16x4                      = svtgpu_aom_variance16x4;
    svt_aom_variance16x64                     = svtgpu_aom_variance16x64;
    svt_aom_variance16x8                      = svtgpu_aom_variance16x8;
    svt_aom_variance32x16                     = svtgpu_aom_variance32x16;
    svt_aom_variance32x32                     = svtgpu_aom_variance32x32;
    svt_aom_variance32x64                     = svtgpu_aom_variance32x64;
    svt_aom_variance32x8                      = svtgpu_aom_variance32x8;
    svt_aom_variance4x16                      = svtgpu_aom_variance4x16;
    svt_aom_variance4x4                       = svtgpu_aom_variance4x4;
    svt_aom_variance4x8                       = svtgpu_aom_variance4x8;
    svt_aom_variance64x128                    = svtgpu_aom_variance64x128;
    svt_aom_variance64x16                     = svtgpu_aom_variance64x16;
    svt_aom_variance64x32                     = svtgpu_aom_variance64x32;
    svt_aom_variance64x64                     = svtgpu_aom_variance64x64;
    svt_aom_variance8x16                      = svtgpu_aom_variance8x16;
    svt_aom_variance8x32                      = svtgpu_aom_variance8x32;
    svt_aom_variance8x4                       = svtgpu_aom_variance8x4;
    svt_aom_variance8x8                       = svtgpu_aom_variance8x8;
    svt_convert_16bit_to_8bit                 = svtgpu_convert_16bit_to_8bit;
    svt_convert_8bit_to_16bit                 = svtgpu_convert_8bit_to_16bit;
    svt_ext_all_sad_calculation_8x8_16x16     = svtgpu_ext_all_sad_calculation_8x8_16x16;
    svt_ext_eight_sad_calculation_32x32_64x64 = svtgpu_ext_eight_sad_calculation_32x32_64x64;
    svt_ext_sad_calculation_32x32_64x64       = svtgpu_ext_sad_calculation_32x32_64x64;
    svt_ext_sad_calculation_8x8_16x16         = svtgpu_ext_sad_calculation_8x8_16x16;
    svt_nxm_sad_kernel                        = svtgpu_nxm_sad_kernel;
    svt_nxm_sad_kernel_sub_sampled            = svtgpu_nxm_sad_kernel_sub_sampled;
    svt_pme_sad_loop_kernel                   = svtgpu_pme_sad_loop_kernel;
    sad_16b_kernel                            = svtgpu_sad_16b_kernel;
    svt_sad_loop_kernel                       = svtgpu_sad_loop_kernel;
}
#endif /* SVTGPU_RTCD_H */
