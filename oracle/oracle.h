/*
 * oracle.h — CPU restatement of the reference's CDEF + deblocking hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code, and
 * only as the checker / CPU baseline — never as the product path.  Each function cites the
 * reference file:line it restates (paths relative to Source/Lib/ of
 * GabrielGao0310/SVT-av1_pro-anchor-v2.1.0-).  Pinned against golden vectors produced by the
 * reference's own C functions (oracle/ref.mk → tests/golden/).
 */
#ifndef SVTGPU_ORACLE_H
#define SVTGPU_ORACLE_H
#include <stdint.h>
#include "../include/svtgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_CDEF_BSTRIDE 144 /* ALIGN_POWER_OF_TWO(128 + 2*8, 3), EbCdef.h:35 */
#define OR_CDEF_VBORDER 3
#define OR_CDEF_HBORDER 8
#define OR_CDEF_VERY_LARGE 0x7F7F
#define OR_CDEF_INBUF_SIZE (OR_CDEF_BSTRIDE * (128 + 2 * OR_CDEF_VBORDER))

/* host-side picture view (plane pointers at the visible origin, strides in samples) */
typedef struct OracleFrame {
    int32_t width, height, bit_depth;
    void   *plane[3];
    int32_t stride[3];
} OracleFrame;

/* ---- kernel level (same signatures/semantics as the reference C functions) ---- */
uint8_t  oracle_cdef_find_dir(const uint16_t *img, int32_t stride, int32_t *var, int32_t coeff_shift);
void     oracle_cdef_filter_block(uint8_t *dst8, uint16_t *dst16, int32_t dstride, const uint16_t *in,
                                  int32_t pri_strength, int32_t sec_strength, int32_t dir, int32_t pri_damping,
                                  int32_t sec_damping, int32_t bsize, int32_t coeff_shift, uint8_t subsampling_factor);
uint64_t oracle_compute_cdef_dist_16bit(const uint16_t *dst, int32_t dstride, const uint16_t *src,
                                        const SvtGpuCdefList *dlist, int32_t cdef_count, int32_t bsize,
                                        int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
uint64_t oracle_compute_cdef_dist_8bit(const uint8_t *dst, int32_t dstride, const uint8_t *src,
                                       const SvtGpuCdefList *dlist, int32_t cdef_count, int32_t bsize,
                                       int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
uint64_t oracle_search_one_dual(int *lev0, int *lev1, int nb_strengths, uint64_t **mse[2], int sb_count,
                                int start_gi, int end_gi);

/* ---- frame level ---- */
int oracle_cdef_controls_for_level(int cdef_level, SvtGpuCdefControls *c);
/* mse: [2][nfb][64], skip: [nfb], dir: [nfb][64], var: [nfb][64]; block_mask as in svtgpu.h (NULL=all) */
int oracle_cdef_search_frame_sb(const OracleFrame *recon, const OracleFrame *src, const uint8_t *block_mask,
                                const uint8_t *fb_bsize, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                                uint64_t *mse, uint8_t *skip, uint8_t *dir_out, int32_t *var_out);
int oracle_cdef_search_frame(const OracleFrame *recon, const OracleFrame *src, const uint8_t *block_mask,
                             const SvtGpuCdefControls *ctrls, int32_t base_q_idx, uint64_t *mse, uint8_t *skip,
                             uint8_t *dir, int32_t *var);
int oracle_cdef_pick(int32_t width, int32_t height, const uint64_t *mse, const uint8_t *skip,
                     const SvtGpuCdefControls *ctrls, int32_t base_q_idx, uint64_t lambda,
                     SvtGpuCdefParams *params, int8_t *fb_strength);
int oracle_cdef_apply_frame(const OracleFrame *recon, OracleFrame *out, const uint8_t *block_mask,
                            const uint8_t *dir, const int32_t *var, const SvtGpuCdefParams *params,
                            const int8_t *fb_strength);

/* ---- deblocking (dlf_oracle.c) ---- */
/* one 4-sample edge segment: vertical = filter across a vertical edge; len in {4, 6, 8, 14} */
void oracle_lpf(uint8_t *s, int32_t pitch, int vertical, int len, const uint8_t *blimit, const uint8_t *limit,
                const uint8_t *thresh);
void oracle_highbd_lpf(uint16_t *s, int32_t pitch, int vertical, int len, const uint8_t *blimit,
                       const uint8_t *limit, const uint8_t *thresh, int32_t bd);
/* mi: [mi_rows][mi_cols] with mi_cols = ((w+7)&~7)/4; filters planes [plane_start, plane_end) in place */
int oracle_dlf_frame(OracleFrame *f, const SvtGpuLfMi *mi, const SvtGpuLfParams *p, int plane_start, int plane_end);
/* the same on a coded-size frame whose unpadded size is crop_w x crop_h (edges at or past it are not filtered) */
int oracle_dlf_frame_crop(OracleFrame *f, const SvtGpuLfMi *mi, const SvtGpuLfParams *p, int plane_start, int plane_end,
                          int crop_w, int crop_h);
/* level search; p in = last-frame levels (already averaged when dlf_avg), out = picked levels */
int oracle_dlf_pick(OracleFrame *recon, const OracleFrame *src, const SvtGpuLfMi *mi, SvtGpuLfParams *p, int dlf_avg,
                    int dlf_avg_uv, int temporal_layer_index, int early_exit, int only4x4);

/* ---- mode-decision distortion (md_oracle.c) ---- */
uint32_t oracle_sad(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h);
uint32_t oracle_sad16(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h);
uint32_t oracle_variance(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h, uint32_t *sse);
uint32_t oracle_highbd_10_variance(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h, uint32_t *sse);
int64_t  oracle_sse(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h);
int64_t  oracle_sse16(const uint16_t *a, int as, const uint16_t *b, int bs, int w, int h);
/* out: [nsb][nref][3][SVTGPU_MD_BLOCKS]; mv: [nsb][nref][2] */
int oracle_md_dist_batch(const OracleFrame *src, const OracleFrame *const *refs, int nref, const int16_t *mv,
                         uint32_t *out);

/* ---- loop restoration (lr_oracle.c) ---- */
void oracle_wiener_round(int bd, int *round0, int *round1);
/* src/dst at the output origin; src readable at rows -3..h+3, cols -3..w+4 */
void oracle_wiener_convolve(const uint16_t *src, int sstride, uint16_t *dst, int dstride, const int16_t *fx,
                            const int16_t *fy, int w, int h, int round0, int round1, int bd);
/* dgd readable at rows -3..h+2, cols -3..w+2 */
void oracle_sgr_filter(const int32_t *dgd, int stride, int w, int h, int eps, int bd, int32_t *flt0, int32_t *flt1,
                       int fstride);
void oracle_decode_xq(const int32_t *xqd, int32_t *xq, int eps);
void oracle_sgr_apply(const uint16_t *dat, int stride, int w, int h, int eps, const int32_t *xqd, uint16_t *dst,
                      int dstride, int bd);
int  oracle_lr_units(int size, int extent);
int  oracle_lr_apply_frame(const OracleFrame *dlf, const OracleFrame *cdef, OracleFrame *out, const int *frame_type,
                           const int *unit_size, const SvtGpuRestUnit *const *units);

/* ---- loop-restoration search (lr_search_oracle.c) ---- */
int oracle_lr_controls_for_level(int wn, int sg, SvtGpuLrSearchControls *c);
int oracle_lr_search_frame(const OracleFrame *recon, const OracleFrame *source, const int *unit_size,
                           const SvtGpuLrSearchControls *c, int *frame_type_out, SvtGpuRestUnit *const *units_out,
                           SvtGpuLrUnitSearch *const *search_out);
/* measurement probe (scripts/r5/sgr_prune_probe.py): per luma unit and ep, search_sgr's exact error and the
 * rounding lower bound; returns the number of units */
int oracle_lr_sgr_probe(const uint16_t *dgd, int dgd_stride, const uint16_t *src, int src_stride, int W, int H, int bd,
                        int usz, int start, int end, int inc, int refine, int64_t *err_out, double *bound_out);

#ifdef __cplusplus
}
#endif
#endif
