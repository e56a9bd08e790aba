/*
 * svtgpu.h — C ABI of the MI355X (gfx950) in-loop-filter / distortion library.
 *
 * Drop-in boundary for SVT-AV1 v2.1.0 (reference: GabrielGao0310/SVT-av1_pro-anchor-v2.1.0-).
 * Two layers, both plain C (no HIP or torch types in any signature):
 *
 *  1. RTCD-compatible per-block entry points.  Each has EXACTLY the signature of the reference's
 *     RTCD function pointer it can be assigned to after svt_aom_setup_common_rtcd_internal /
 *     svt_aom_setup_rtcd_internal (Source/Lib/Encoder/Globals/EbEncHandle.c:1530-1531).  They take
 *     host pointers, run the HIP kernel on the library's default device and return the result
 *     synchronously.  They exist for unit parity (the reference's own gtests call these pointers);
 *     they are far too fine-grained to be fast.
 *
 *  2. Frame-level entry points (the real GPU boundary).  They replace the reference's C loops over
 *     64x64 filter blocks (cdef_seg_search, finish_cdef_search, svt_av1_cdef_frame, ...) and run on
 *     device-resident frames.  Every call takes a `void *stream` (a hipStream_t; NULL = the
 *     context's own stream) and is asynchronous with respect to the host unless stated otherwise.
 *
 * Error convention: functions returning int return SVTGPU_OK (0) or a negative SVTGPU_ERR_* code;
 * nothing throws or longjmps across this ABI.  Per-block shims cannot report errors through their
 * reference signature; they abort() with a message if the device is missing (the encoder must not
 * install them without a device — see svtgpu_device_available()).
 */
#ifndef SVTGPU_H
#define SVTGPU_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVTGPU_OK 0
#define SVTGPU_ERR_INVALID_ARG (-1)
#define SVTGPU_ERR_HIP (-2)
#define SVTGPU_ERR_UNSUPPORTED (-3)
#define SVTGPU_ERR_NO_DEVICE (-4)
#define SVTGPU_ERR_OOM (-5)

/* Block-size codes used by the per-block CDEF shims; values equal the reference's BlockSize enum
 * (Source/Lib/Common/Codec/EbDefinitions.h:769-772). */
#define SVTGPU_BLOCK_4X4 0
#define SVTGPU_BLOCK_4X8 1
#define SVTGPU_BLOCK_8X4 2
#define SVTGPU_BLOCK_8X8 3

/* Layout-identical to the reference's CdefList (EbDefinitions.h:253-256). */
typedef struct SvtGpuCdefList {
    uint8_t by;
    uint8_t bx;
} SvtGpuCdefList;

/* Layout-identical to the reference's SgrParamsType (EbDefinitions.h:1768-1771): radii and s values of an ep. */
typedef struct SvtGpuSgrParams {
    int32_t r[2];
    int32_t s[2];
} SvtGpuSgrParams;

/* Layout-identical to the reference's ConvolveParams (EbDefinitions.h:577-590); the Wiener shims read
 * round_0 / round_1 only. */
typedef struct SvtGpuConvolveParams {
    int32_t  ref;
    int32_t  do_average;
    void    *dst;
    int32_t  dst_stride;
    int32_t  round_0;
    int32_t  round_1;
    int32_t  plane;
    int32_t  is_compound;
    int32_t  use_jnt_comp_avg;
    int32_t  fwd_offset;
    int32_t  bck_offset;
    int32_t  use_dist_wtd_comp_avg;
} SvtGpuConvolveParams;

/* Type hooks for a C translation unit compiled against the reference's own headers (INTEGRATION.md §2;
 * oracle/ref_harness/rtcd_bind.c): defining these to CdefList, BlockSize, SgrParamsType, ConvolveParams and
 * EbBitDepth before including this header makes the shim prototypes name the reference's types, so every shim
 * assigns to its RTCD function pointer without a cast.  The layouts are identical, so the ABI is the same. */
#ifndef SVTGPU_CDEF_LIST_T
#define SVTGPU_CDEF_LIST_T SvtGpuCdefList
#endif
#ifndef SVTGPU_BLOCK_SIZE_T
#define SVTGPU_BLOCK_SIZE_T int32_t
#endif
#ifndef SVTGPU_SGR_PARAMS_T
#define SVTGPU_SGR_PARAMS_T SvtGpuSgrParams
#endif
#ifndef SVTGPU_CONVOLVE_PARAMS_T
#define SVTGPU_CONVOLVE_PARAMS_T SvtGpuConvolveParams
#endif
#ifndef SVTGPU_BIT_DEPTH_T
#define SVTGPU_BIT_DEPTH_T int32_t
#endif

/* ---------------------------------------------------------------------------------------------
 * Library / device
 * ------------------------------------------------------------------------------------------- */
/* 1 when a gfx950 device is visible and the kernels are loadable, else 0. Never aborts. */
int         svtgpu_device_available(void);
const char *svtgpu_version(void);
/* ABI revision of this header: bumped whenever a struct passed across the boundary changes layout or an entry
 * point changes meaning (6: SvtGpuLrProfile::ms_events, svtgpu_comm_create_bounded, the asynchronous LR search
 * svtgpu_lr_search_frame_async; 7: svtgpu_cdef_apply_frame accepts params == NULL, svtgpu_stream_create; 8: the CCSO entry points,
 * SvtGpuCcsoParams).
 * A caller built against another header checks svtgpu_abi_version() ==
 * SVTGPU_ABI_VERSION once at start-up and refuses to run on a mismatch. */
#define SVTGPU_ABI_VERSION 8
int32_t     svtgpu_abi_version(void);
const char *svtgpu_error_string(int code);

typedef struct SvtGpuContext SvtGpuContext;
/* One context per (process, device). Owns a HIP stream and the scratch of the frame-level calls. */
int   svtgpu_context_create(int device, SvtGpuContext **out);
void  svtgpu_context_destroy(SvtGpuContext *ctx);
void *svtgpu_context_stream(SvtGpuContext *ctx); /* the context's hipStream_t */
int   svtgpu_synchronize(SvtGpuContext *ctx, void *stream);
/* A stream for the frame-level calls (a hipStream_t; priority > 0 the device's highest, < 0 its lowest, 0 normal).
 * Each stream is one hardware queue while the process has no more streams than GPU_MAX_HW_QUEUES; past that, streams
 * share queues and a frame's chain waits behind another's.  An encoder running several pictures at once creates its
 * per-picture streams here (or otherwise exactly as many as it runs), not from a framework's stream pool (round 6:
 * torch.cuda.Stream()'s pool of 32 streams per priority cost 1080p 10-bit at four frames in flight 23%). */
int  svtgpu_stream_create(SvtGpuContext *ctx, int32_t priority, void **out_stream);
void svtgpu_stream_destroy(void *stream);
/* Plain device buffers for the pointer-level entry points (CCSO, svtgpu_convert_plane, ...) when the caller has no
 * allocator of its own; upload / download are complete when they return (the stream is synchronized). */
int  svtgpu_buffer_alloc(SvtGpuContext *ctx, size_t bytes, void **dev_out);
void svtgpu_buffer_free(void *dev);
int  svtgpu_buffer_upload(void *dev, const void *host, size_t bytes, void *stream);
int  svtgpu_buffer_download(void *host, const void *dev, size_t bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Device-resident 4:2:0 pictures
 *   Samples are uint8 when bit_depth == 8 and uint16 when bit_depth == 10 (the reference's
 *   "16-bit pipeline", EbEncHandle.c:4534).  width/height are luma sizes, multiples of 8.
 *   Plane p (0=Y,1=U,2=V) is stored with stride svtgpu_frame_stride(f, p) samples and no padding
 *   requirement on the caller side.
 * ------------------------------------------------------------------------------------------- */
typedef struct SvtGpuFrame SvtGpuFrame;
int      svtgpu_frame_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t bit_depth,
                             SvtGpuFrame **out);
void     svtgpu_frame_destroy(SvtGpuFrame *f);
int32_t  svtgpu_frame_stride(const SvtGpuFrame *f, int plane);
void    *svtgpu_frame_plane_ptr(SvtGpuFrame *f, int plane); /* device pointer */
/* host <-> device copies of one plane; host_stride in samples. Asynchronous on `stream` unless the
 * host buffer is pageable (then HIP makes it synchronous). */
int svtgpu_frame_upload(SvtGpuFrame *f, int plane, const void *host, int32_t host_stride, void *stream);
int svtgpu_frame_download(const SvtGpuFrame *f, int plane, void *host, int32_t host_stride, void *stream);
/* Only the samples of rect = {x0, y0, x1, y1} (plane coordinates) of one plane; `host` is the plane's origin as for
 * svtgpu_frame_upload.  A rank of a tiled picture uploads its SvtGpuTilePlan::in_rect (chroma halved, outward). */
int svtgpu_frame_upload_rect(SvtGpuFrame *f, int plane, const void *host, int32_t host_stride, const int32_t rect[4],
                             void *stream);
int svtgpu_frame_copy(SvtGpuFrame *dst, const SvtGpuFrame *src, void *stream);

/* ---------------------------------------------------------------------------------------------
 * A picture tiled over several GPUs (BASELINE.json config 4).  No reference counterpart: the
 * reference splits a picture into segments for its worker threads (cdef_seg_search / restoration_seg_search per
 * segment, EbEncHandle.c:503-514) and gathers their results under a mutex (EbCdefProcess.c:406, EbRestProcess.c:614).
 * Here each rank (one process per GPU) takes a tile, and the frame-level calls exchange what the reference's
 * gather hands to its sequential finish: the DLF trial SSEs, the CDEF search tables and the LR search records.
 * ------------------------------------------------------------------------------------------- */
#define SVTGPU_COMM_ID_BYTES 128
typedef struct SvtGpuComm SvtGpuComm;
/* RCCL over xGMI: rank 0 creates the id, the caller broadcasts its bytes (any transport), every rank creates its
 * communicator on its device.  One communicator per frame in flight. */
int svtgpu_comm_unique_id(uint8_t id[SVTGPU_COMM_ID_BYTES]);
int svtgpu_comm_create(SvtGpuContext *ctx, int32_t nranks, int32_t rank, const uint8_t id[SVTGPU_COMM_ID_BYTES],
                       SvtGpuComm **out);
/* svtgpu_comm_create with a bounded init: the communicator is created non-blocking (ncclCommInitRankConfig, blocking
 * = 0) and polled against timeout_ms (0: the default deadline, SVTGPU_COMM_TIMEOUT_MS or 60000 ms).  A peer that never
 * joins (it died between the id broadcast and its init) returns SVTGPU_ERR_HIP within the deadline with
 * svtgpu_error_string naming "communicator init", the frame slot `slot`, this rank and the rank count; the partial
 * communicator is aborted.  svtgpu_comm_create = this with timeout_ms 0 and slot -1.  SVTGPU_COMM_INIT=blocking
 * restores the blocking ncclCommInitRank. */
int svtgpu_comm_create_bounded(SvtGpuContext *ctx, int32_t nranks, int32_t rank, const uint8_t id[SVTGPU_COMM_ID_BYTES],
                               int32_t timeout_ms, int32_t slot, SvtGpuComm **out);
/* A caller-supplied host transport (e.g. MPI or gloo): allreduce_u64 sums n uint64 element-wise over the ranks in
 * place (every rank receives the sums) and returns 0.  Device buffers are staged through pinned host memory.  For
 * rehearsals on CPUs and for several ranks on one GPU (RCCL needs one rank per device). */
typedef struct SvtGpuHostTransport {
    void *user;
    int (*allreduce_u64)(void *user, uint64_t *buf, size_t n);
} SvtGpuHostTransport;
int     svtgpu_comm_create_host(int32_t nranks, int32_t rank, const SvtGpuHostTransport *t, SvtGpuComm **out);
void    svtgpu_comm_destroy(SvtGpuComm *c);
int32_t svtgpu_comm_nranks(const SvtGpuComm *c);
int32_t svtgpu_comm_rank(const SvtGpuComm *c);
/* element-wise sum of n uint64 over the ranks, in place; on_device: buf is device memory (enqueued on `stream` with
 * RCCL), else host memory (synchronous) */
int svtgpu_comm_allreduce_u64(SvtGpuComm *c, void *buf, size_t n, int32_t on_device, void *stream);
/* Every exchange is bounded by the communicator's deadline (default 60000 ms, SVTGPU_COMM_TIMEOUT_MS overrides it).
 * A frame-level call whose exchange does not complete in time (a peer rank skipped it, or failed before reaching it)
 * returns SVTGPU_ERR_HIP, svtgpu_error_string names the exchange ("DLF trial SSEs", "CDEF search tables", "LR search
 * records"), the frame slot and the exchange's sequence number; an RCCL communicator is aborted (ncclCommAbort ends
 * this rank's pending collectives) and the communicator fails every later call (svtgpu_comm_failed).  A host
 * transport bounds its own wait by svtgpu_comm_timeout_ms and returns non-zero when it expires. */
int     svtgpu_comm_set_timeout(SvtGpuComm *c, int32_t timeout_ms);
int32_t svtgpu_comm_timeout_ms(const SvtGpuComm *c);
int     svtgpu_comm_set_slot(SvtGpuComm *c, int32_t frame_slot); /* the frame slot named in a timeout's message */
int32_t svtgpu_comm_failed(const SvtGpuComm *c);
/* host wait for `stream`, bounded by the deadline when one of the communicator's device-side exchanges (enqueued
 * without a host wait: svtgpu_comm_allreduce_u64 on device memory) was enqueued on `stream` since its last completed
 * wait -- the whole wait is then bounded (per-exchange completion markers lengthened a tiled rank's latency chains
 * by 7 %), so work queued behind an exchange counts against the deadline too */
int     svtgpu_comm_sync(SvtGpuComm *c, void *stream);
/* the number of per-block RTCD shim calls this process made (each runs on the process-wide default context): evidence
 * that an encoder with the shims installed really ran its kernels on the device */
uint64_t svtgpu_shim_calls(void);
/* test support: holds `stream` busy for `ms` milliseconds (<= 10000) with one spinning wave */
int     svtgpu_debug_stall(SvtGpuContext *ctx, void *stream, int32_t ms);

/* The tiles of a gx x gy split of a width x height picture and what rank `rank` (row-major) computes.  Tile edges
 * fall on the luma restoration-unit grid (unit_size[0], a multiple of 64: also filter-block and superblock edges), so
 * each rank's loop-restoration units lie in its own part of the frame:
 *   tile       {x0, y0, x1, y1} luma: the rank's share of the DLF trial SSEs (a partition of the frame);
 *   fb_rect    {col0, row0, col1, row1}: the 64x64 CDEF filter blocks it searches (a partition);
 *   lr_units   per plane {col0, row0, col1, row1} unit indices it searches (a partition of each plane's units);
 *   lr_out     per plane {x0, y0, x1, y1} plane samples: the union of those units, the part of the final picture the
 *              rank produces (a partition);
 *   cdef_out   {x0, y0, x1, y1} luma: the CDEF output its LR search and apply read (lr_out plus an 8-sample apron);
 *   dlf_out    {x0, y0, x1, y1} luma: the DLF output its CDEF search / apply and LR boundary lines read (its tile and
 *              lr_out plus a 16-sample apron);
 *   in_rect    {x0, y0, x1, y1} luma: the recon and source samples the rank's calls read (dlf_out plus the deblocking
 *              filter's 16-sample reach): what a rank uploads of each input picture.
 * Host only.  SVTGPU_ERR_INVALID_ARG when some rank would get no unit. */
typedef struct SvtGpuTilePlan {
    int32_t tile[4], fb_rect[4], lr_units[3][4], lr_out[3][4], cdef_out[4], dlf_out[4], in_rect[4];
} SvtGpuTilePlan;
int svtgpu_tile_plan(int32_t width, int32_t height, const int32_t unit_size[3], int32_t gx, int32_t gy, int32_t rank,
                     SvtGpuTilePlan *out);
/* The same for a picture of sb_size (64 or 128) superblocks: with 128 the tile edges are also multiples of 128, so no
 * 128x128 CDEF area is cut (svtgpu_tile_plan = sb_size 64). */
int svtgpu_tile_plan_sb(int32_t width, int32_t height, const int32_t unit_size[3], int32_t sb_size, int32_t gx,
                        int32_t gy, int32_t rank, SvtGpuTilePlan *out);
/* A picture whose crop size (frm_size.frame_width x frame_height, the area loop restoration covers) is below its
 * 8-aligned coded size (width x height: the deblocking / CDEF frames, coded - crop < 8 each way): the restoration
 * units tile the crop (chroma rounded up), the tiles keep their edges on the luma unit grid and the last tile runs to
 * the coded edge.  Each rank's LR state is created with the crop size and its DLF state told the crop
 * (svtgpu_dlf_set_crop), as on one GPU.  svtgpu_tile_plan_sb = crop equal to the coded size. */
int svtgpu_tile_plan_crop(int32_t width, int32_t height, int32_t crop_w, int32_t crop_h, const int32_t unit_size[3],
                          int32_t sb_size, int32_t gx, int32_t gy, int32_t rank, SvtGpuTilePlan *out);

/* ---------------------------------------------------------------------------------------------
 * CDEF — per-block RTCD shims (host pointers, synchronous)
 * ------------------------------------------------------------------------------------------- */
/* replaces svt_aom_cdef_find_dir (common_dsp_rtcd.h:1017); C: EbCdef.c:150 */
uint8_t svtgpu_cdef_find_dir(const uint16_t *img, int32_t stride, int32_t *var, int32_t coeff_shift);
/* replaces svt_aom_cdef_find_dir_dual (common_dsp_rtcd.h:1096); C: EbCdef.c:212 */
void svtgpu_cdef_find_dir_dual(const uint16_t *img1, const uint16_t *img2, int stride, int32_t *var1,
                               int32_t *var2, int32_t coeff_shift, uint8_t *out1, uint8_t *out2);
/* replaces svt_cdef_filter_block (common_dsp_rtcd.h:1099); C: EbCdef.c:253.
 * `in` points into a CDEF_BSTRIDE(=144)-stride buffer; rows -2..h+1 and cols -2..w+1 are read. */
void svtgpu_cdef_filter_block(uint8_t *dst8, uint16_t *dst16, int32_t dstride, const uint16_t *in,
                              int32_t pri_strength, int32_t sec_strength, int32_t dir, int32_t pri_damping,
                              int32_t sec_damping, int32_t bsize, int32_t coeff_shift,
                              uint8_t subsampling_factor);
/* replaces svt_compute_cdef_dist_16bit / _8bit (aom_dsp_rtcd.h:62-64); C: EbEncCdef.c:129/175 */
uint64_t svtgpu_compute_cdef_dist_16bit(const uint16_t *dst, int32_t dstride, const uint16_t *src,
                                        const SVTGPU_CDEF_LIST_T *dlist, int32_t cdef_count, SVTGPU_BLOCK_SIZE_T bsize,
                                        int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
uint64_t svtgpu_compute_cdef_dist_8bit(const uint8_t *dst8, int32_t dstride, const uint8_t *src8,
                                       const SVTGPU_CDEF_LIST_T *dlist, int32_t cdef_count, SVTGPU_BLOCK_SIZE_T bsize,
                                       int32_t coeff_shift, int32_t pli, uint8_t subsampling_factor);
/* replaces svt_search_one_dual (aom_dsp_rtcd.h:239); C: EbEncCdef.c:627 */
uint64_t svtgpu_search_one_dual(int *lev0, int *lev1, int nb_strengths, uint64_t **mse[2], int sb_count,
                                int start_gi, int end_gi);
/* replaces svt_cdef_filter_block_8xn_16 (common_dsp_rtcd.h:1100; AVX2 only in the reference,
 * cdef_block_avx2.c:463): an 8-wide luma block, rows 0, s, 2s, ... (s = subsampling_factor) of `height`, into a
 * uint16 dst; `in` points into a CDEF_BSTRIDE(=144)-stride buffer, pri_strength already adjusted */
void svtgpu_cdef_filter_block_8xn_16(const uint16_t *const in, const int32_t pri_strength, const int32_t sec_strength,
                                     const int32_t dir, int32_t pri_damping, int32_t sec_damping,
                                     const int32_t coeff_shift, uint16_t *const dst, const int32_t dstride,
                                     uint8_t height, uint8_t subsampling_factor);
/* replaces svt_aom_copy_rect8_8bit_to_16bit (common_dsp_rtcd.h:1105; C EbCdef.c:303): the 8-bit -> 16-bit
 * staging copy of the CDEF input buffer, v rows x h columns */
void svtgpu_aom_copy_rect8_8bit_to_16bit(uint16_t *dst, int32_t dstride, const uint8_t *src, int32_t sstride, int32_t v,
                                         int32_t h);

/* ---------------------------------------------------------------------------------------------
 * CDEF — frame level (device-resident)
 * ------------------------------------------------------------------------------------------- */
#define SVTGPU_CDEF_TOTAL_STRENGTHS 64
#define SVTGPU_CDEF_MAX_STRENGTHS 16

/* Subset of the reference's CdefControls (EbPictureControlSet.h:592-628) that the search and pick
 * read.  Strength codes are pri*4 + sec (sec code 3 means strength 4), as in
 * EncModeConfig.c:860-1330. */
typedef struct SvtGpuCdefControls {
    uint8_t  first_pass_fs_num;
    uint8_t  default_second_pass_fs_num;
    uint8_t  default_first_pass_fs[SVTGPU_CDEF_TOTAL_STRENGTHS];
    uint8_t  default_second_pass_fs[SVTGPU_CDEF_TOTAL_STRENGTHS];
    int8_t   default_first_pass_fs_uv[SVTGPU_CDEF_TOTAL_STRENGTHS];  /* -1 = chroma not tested */
    int8_t   default_second_pass_fs_uv[SVTGPU_CDEF_TOTAL_STRENGTHS]; /* -1 = chroma not tested */
    uint8_t  subsampling_factor;                                     /* 1, 2 or 4 */
    uint16_t zero_fs_cost_bias;                                      /* 0 = off, else x/64 */
    /* use_reference_cdef_fs levels (11, 14, 15, 17): no strength search; the frame uses the strength pair the
     * mode-decision configuration predicted from the references (pred_y_f / pred_uv_f, strength codes 0..63,
     * set by the caller as EbModeDecisionConfigurationProcess.c:765-840 does) */
    int8_t   use_reference_cdef_fs;
    int8_t   pred_y_f;
    int8_t   pred_uv_f;
} SvtGpuCdefControls;

/* Fill `c` exactly as set_cdef_controls(cdef_level) does (EncModeConfig.c:860-1330), levels 1..17
 * (pred_y_f / pred_uv_f left 0). Returns SVTGPU_ERR_UNSUPPORTED for level 0 (CDEF off).
 * fast_decode/resolution tweaks of the zero_fs_cost_bias are applied by the caller. */
int svtgpu_cdef_controls_for_level(int cdef_level, SvtGpuCdefControls *c);

/* Frame parameters chosen by the pick; layout mirrors CdefParams (EbAv1Structs.h:359-369). */
typedef struct SvtGpuCdefParams {
    uint8_t cdef_damping;
    uint8_t cdef_bits;
    uint8_t cdef_y_strength[SVTGPU_CDEF_MAX_STRENGTHS];
    uint8_t cdef_uv_strength[SVTGPU_CDEF_MAX_STRENGTHS];
} SvtGpuCdefParams;

/* Device-resident search state for one frame (mse_seg, skip_cdef_seg and cdef_dir_data of the
 * reference's PictureControlSet, EbPictureControlSet.h:268-270). */
typedef struct SvtGpuCdefFrameState SvtGpuCdefFrameState;
int  svtgpu_cdef_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuCdefFrameState **out);
void svtgpu_cdef_state_destroy(SvtGpuCdefFrameState *s);
int32_t svtgpu_cdef_state_nfb(const SvtGpuCdefFrameState *s); /* nvfb*nhfb */

/* Per-8x8 "filter this block" mask, row-major, ((h+7)/8) x ((w+7)/8) bytes; an 8x8 block is
 * listed iff any of its four 4x4 mode-info units is non-skip (svt_sb_compute_cdef_list,
 * EbEncCdef.c:238).  Upload once per frame; NULL mask = every block listed. */
int svtgpu_cdef_set_block_mask(SvtGpuCdefFrameState *s, const uint8_t *host_mask, void *stream);

/* SB128 mode info: the BlockSize (EbDefinitions.h enum; 13 = 64X128, 14 = 128X64, 15 = 128X128) of the mode
 * info at each 64x64 filter block's top-left, nfb bytes row-major — what cdef_seg_search and finish_cdef_search
 * read (EbCdefProcess.c:188-199, EbEncCdef.c:805-812).  The search then folds each 128-wide area into its top-left
 * filter block and the pick copies the area's strength into the other halves.  NULL = 64x64 superblocks.
 * With frame bands (svtgpu_cdef_set_fb_rows) the band edges must fall on even filter-block rows. */
int svtgpu_cdef_set_fb_bsize(SvtGpuCdefFrameState *s, const uint8_t *fb_bsize, void *stream);

/* ≙ all segments of cdef_seg_search (EbCdefProcess.c:114-357).  recon = DLF output, source = input picture
 * (same geometry/bit depth).  With use_reference_cdef_fs no strength is searched (EbCdefProcess.c:400): only
 * the per-8x8 directions/variances the apply needs are computed (svt_av1_cdef_frame finds them itself then,
 * EbEncCdef.c:403), and the mse table is zeroed. */
int svtgpu_cdef_search_frame(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                             const SvtGpuCdefControls *ctrls, int32_t base_q_idx, void *stream);

/* ≙ finish_cdef_search (EbEncCdef.c:728-926) with svt_search_one_dual on the device; with
 * use_reference_cdef_fs its first branch (:744-789): one strength pair {pred_y_f, pred_uv_f}, index 0 everywhere.
 * lambda = full_lambda of the frame (computed by the encoder's lambda function table).
 * Writes params and the per-FB strength index (int8 per FB, host array of nfb entries) and keeps
 * the per-FB index on the device for svtgpu_cdef_apply_frame.  Synchronous (returns host data). */
int svtgpu_cdef_pick(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                     uint64_t lambda, SvtGpuCdefParams *params_out, int8_t *fb_strength_out, void *stream);

/* The same pick with no host wait (round 6): the settle check's outcome reaches the later strength-search steps
 * through device memory (they exit at once when every chain has settled), and the RD choice leaves the frame
 * parameters and the per-FB indices in device memory, where svtgpu_cdef_apply_frame(params = NULL) reads them --
 * everything in stream order.  svtgpu_cdef_read_params returns them (after a bounded wait for `stream`) once the
 * caller needs them on the host, e.g. to write the frame header. */
int svtgpu_cdef_pick_async(SvtGpuCdefFrameState *s, const SvtGpuCdefControls *ctrls, int32_t base_q_idx,
                           uint64_t lambda, void *stream);
int svtgpu_cdef_read_params(SvtGpuCdefFrameState *s, SvtGpuCdefParams *params_out, int8_t *fb_strength_out,
                            void *stream);

/* Optional override of the per-FB strength index used by apply (host array of nfb entries). */
int svtgpu_cdef_set_fb_strength(SvtGpuCdefFrameState *s, const int8_t *fb_strength, void *stream);

/* ≙ svt_av1_cdef_frame (EbEncCdef.c:284-610): apply params to `recon` (DLF output) and write the
 * filtered picture to `out` (out-of-place; the reference's in-place result with its saved
 * unfiltered line/column buffers is identical).  Uses dir/var of the last search.  params == NULL: the parameters
 * of the last svtgpu_cdef_pick_async, read from device memory in stream order. */
int svtgpu_cdef_apply_frame(SvtGpuCdefFrameState *s, const SvtGpuFrame *recon, SvtGpuFrame *out,
                            const SvtGpuCdefParams *params, void *stream);

/* Frame tiling across GPUs (BASELINE config 4): restrict search and apply to filter-block rows
 * [fb_row_begin, fb_row_end).  Samples outside the band are still read as filter context (apron), so
 * the picture passed in must hold valid samples for the band +-3 rows.  Default: all rows. */
int svtgpu_cdef_set_fb_rows(SvtGpuCdefFrameState *s, int32_t fb_row_begin, int32_t fb_row_end);
/* A picture tiled over GPUs (svtgpu_tile_plan): the search covers the filter blocks of fb_rect = {col0, row0, col1,
 * row1} only and leaves zeros elsewhere in the tables; svtgpu_cdef_pick first sums the mse / skip / dir / var tables
 * over `comm` (one contributor per entry: the gather of every rank's blocks; the pick is then the same on every rank;
 * the sums run once per search: a second pick on the same search reads the gathered tables); the apply writes only the luma rectangle out_rect = {x0, y0, x1, y1} (chroma halved, rounded outward), reading
 * the DLF output 2 samples around it.  NULL rects: the whole frame; NULL comm: no exchange. */
int svtgpu_cdef_set_tile(SvtGpuCdefFrameState *s, const int32_t fb_rect[4], const int32_t out_rect[4],
                         SvtGpuComm *comm);
/* Use caller-owned device memory for the search tables: mse [2][nfb][64] uint64 and skip [nfb] uint8
 * (e.g. buffers all-reduced with RCCL between the search and the pick).  NULL, NULL restores the
 * state's own buffers.  svtgpu_cdef_clear_tables zeroes both (a band search then leaves zeros —
 * the identity of an all-reduce-sum — outside its rows).  The library touches exactly nfb bytes of a
 * bound skip table (the tiled pick sums it through a padded copy of its own). */
int svtgpu_cdef_bind_tables(SvtGpuCdefFrameState *s, void *mse_dev, void *skip_dev);
/* The same for the per-8x8 direction/variance tables the apply reuses: dir [nfb][64] uint8, var [nfb][64]
 * int32 (zero outside a band after svtgpu_cdef_clear_tables, so an all-reduce-sum completes them and every
 * rank can apply the whole frame). */
int svtgpu_cdef_bind_dir_tables(SvtGpuCdefFrameState *s, void *dir_dev, void *var_dev);
/* zeroes mse, skip, dir and var */
int svtgpu_cdef_clear_tables(SvtGpuCdefFrameState *s, void *stream);

/* Host views of the search results (synchronous). mse: [2][nfb][64] uint64, skip: [nfb] uint8,
 * dir: [nfb][64] uint8 and var: [nfb][64] int32 (8x8 blocks of the FB, row-major). Any may be NULL. */
int svtgpu_cdef_read_state(SvtGpuCdefFrameState *s, uint64_t *mse, uint8_t *skip, uint8_t *dir, int32_t *var,
                           void *stream);
/* Device pointer of the [2][nfb][64] uint64 mse table (for RCCL gathers across tiles). */
void *svtgpu_cdef_mse_device_ptr(SvtGpuCdefFrameState *s);

/* ---------------------------------------------------------------------------------------------
 * Deblocking loop filter — per-segment RTCD shims (host pointers, synchronous).
 * Each filters one 4-sample edge segment exactly like the reference C (EbDeblockingCommon.c).
 * ------------------------------------------------------------------------------------------- */
/* replace svt_aom_lpf_{horizontal,vertical}_{4,6,8,14} (common_dsp_rtcd.h:1116-1131) */
void svtgpu_lpf_horizontal_4(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                             const uint8_t *thresh);
void svtgpu_lpf_horizontal_6(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                             const uint8_t *thresh);
void svtgpu_lpf_horizontal_8(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                             const uint8_t *thresh);
void svtgpu_lpf_horizontal_14(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                              const uint8_t *thresh);
void svtgpu_lpf_vertical_4(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                           const uint8_t *thresh);
void svtgpu_lpf_vertical_6(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                           const uint8_t *thresh);
void svtgpu_lpf_vertical_8(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                           const uint8_t *thresh);
void svtgpu_lpf_vertical_14(uint8_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                            const uint8_t *thresh);
/* replace svt_aom_highbd_lpf_{horizontal,vertical}_{4,6,8,14} (common_dsp_rtcd.h:1132-1146) */
void svtgpu_highbd_lpf_horizontal_4(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                    const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_horizontal_6(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                    const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_horizontal_8(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                    const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_horizontal_14(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                     const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_vertical_4(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                  const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_vertical_6(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                  const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_vertical_8(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                  const uint8_t *thresh, int32_t bd);
void svtgpu_highbd_lpf_vertical_14(uint16_t *s, int32_t pitch, const uint8_t *blimit, const uint8_t *limit,
                                   const uint8_t *thresh, int32_t bd);

/* ---------------------------------------------------------------------------------------------
 * Deblocking loop filter — frame level (device-resident, in place)
 * ------------------------------------------------------------------------------------------- */
/* One record per 4x4 mode-info unit (mi), raster order, mi_rows x mi_cols (mi = 4 luma samples;
 * frame dimensions rounded up to 8).  The MbModeInfo fields set_lpf_parameters reads
 * (EbDeblockingFilter.c:162-282); values are the reference's enums (BlockSize, PredictionMode,
 * MvReferenceFrame with INTRA_FRAME = 0). */
typedef struct SvtGpuLfMi {
    uint8_t bsize;      /* block_mi.bsize */
    uint8_t tx_depth;   /* block_mi.tx_depth (0..2) */
    uint8_t skip;       /* block_mi.skip */
    int8_t  ref_frame0; /* block_mi.ref_frame[0] */
    uint8_t mode;       /* block_mi.mode */
    uint8_t segment_id; /* block_mi.segment_id */
    uint8_t pad[2];
} SvtGpuLfMi;

/* Frame loop-filter parameters: struct LoopFilter (EbDefinitions.h:1903-1920) + the segmentation
 * feature arrays (EbSegmentationParams.h:49-53) the level table depends on.  delta_lf is not
 * supported (delta_lf_present = 0). */
typedef struct SvtGpuLfParams {
    int32_t filter_level[2]; /* luma: [0] vertical edges, [1] horizontal edges */
    int32_t filter_level_u;
    int32_t filter_level_v;
    int32_t sharpness_level;
    uint8_t mode_ref_delta_enabled;
    int8_t  ref_deltas[8];
    int8_t  mode_deltas[2];
    uint8_t segmentation_enabled;
    int16_t seg_feature_data[8][8];    /* [segment][SEG_LVL_*] */
    int16_t seg_feature_enabled[8][8]; /* [segment][SEG_LVL_*] */
} SvtGpuLfParams;

typedef struct SvtGpuDlfState SvtGpuDlfState;
int  svtgpu_dlf_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuDlfState **out);
void svtgpu_dlf_state_destroy(SvtGpuDlfState *s);
/* upload the mi grid ((h+7)/8*2 rows x (w+7)/8*2 cols records): asynchronous on `stream` through pinned staging,
 * the caller may reuse its buffer on return (one grid per frame) */
int svtgpu_dlf_set_mode_info(SvtGpuDlfState *s, const SvtGpuLfMi *mi, void *stream);
/* the same from a grid already in device memory (`d_mi`, same layout; e.g. written by a device mode decision):
 * copied in stream order (the caller may overwrite `d_mi` once `stream` has passed this call), no host pass and no
 * PCIe.  The records kernel checks the fields; a grid with records out of range is clamped and reported as
 * SVTGPU_ERR_INVALID_ARG by the next svtgpu_dlf_pick, or by the next svtgpu_dlf_frame(_to) when no pick ran (the
 * FROM_Q levels); each upload is judged on its own. */
int svtgpu_dlf_set_mode_info_device(SvtGpuDlfState *s, const SvtGpuLfMi *d_mi, void *stream);
/* The picture's unpadded size when it is off the 8-sample grid (scs->max_input_luma_width - max_input_pad_right,
 * _height - _pad_bottom; EbDeblockingFilter.c:99-129): set_lpf_parameters filters no edge at or past it in a plane
 * (luma crop_width x crop_height, chroma both >> 1; :173-178), while the frames and the mode-info grid stay the
 * 8-aligned coded size the state was created with.  Default: the coded size.  Takes effect at the next
 * svtgpu_dlf_set_mode_info(_device). */
int svtgpu_dlf_set_crop(SvtGpuDlfState *s, int32_t crop_width, int32_t crop_height);
/* ≙ svt_av1_loop_filter_frame(frame, pcs, plane_start, plane_end) (EbDeblockingFilter.c:624-653):
 * all vertical edges of each plane, then all horizontal edges (equivalent to the reference's
 * SB-lagged order with combine_vert_horz_lf = 1, :41, :580-605), in place on `frame`. */
int svtgpu_dlf_frame(SvtGpuDlfState *s, SvtGpuFrame *frame, const SvtGpuLfParams *params, int32_t plane_start,
                     int32_t plane_end, void *stream);
/* Out-of-place form of svtgpu_dlf_frame: reads `in`, writes every sample of planes
 * [plane_start, plane_end) of `out` (filtered, or copied when the plane is not filtered). */
int svtgpu_dlf_frame_to(SvtGpuDlfState *s, const SvtGpuFrame *in, SvtGpuFrame *out, const SvtGpuLfParams *params,
                        int32_t plane_start, int32_t plane_end, void *stream);
/* ≙ svt_av1_pick_filter_level(LPF_PICK_FROM_FULL_IMAGE) (EbDeblockingFilter.c:1129-1252): bisection
 * on the filter level per plane with a device trial per level (filter + SSE vs `source` + restore).
 * `params` carries the previous levels in and the picked levels out; `recon` is left unfiltered.
 * dlf_avg_uv/temporal_layer_index select the reference's "use averaged chroma levels" shortcut.
 * Synchronous. */
int svtgpu_dlf_pick(SvtGpuDlfState *s, SvtGpuFrame *recon, const SvtGpuFrame *source, SvtGpuLfParams *params,
                    int32_t dlf_avg, int32_t dlf_avg_uv, int32_t temporal_layer_index,
                    int32_t early_exit_convergence, int32_t tx_mode_only_4x4, void *stream);
/* The same level search with no host wait (≙ svt_av1_pick_filter_level, LPF_PICK_FROM_FULL_IMAGE): the bisection of
 * search_filter_level (EbDeblockingFilter.c:886-991) runs on the device -- every trial round's last workgroup takes the
 * step, a final one-workgroup kernel completes a search still open after the rounds enqueued (sized from the previous
 * search) -- and the picked levels stay there.  `params` carries the previous levels in (read at the call).
 * svtgpu_dlf_frame(_to)(..., params = NULL, ...) then filters with the picked levels in stream order, and
 * svtgpu_dlf_read_levels waits for them (the frame header's levels).  A picture tiled over GPUs runs the synchronous
 * search here and keeps its levels. */
int svtgpu_dlf_pick_async(SvtGpuDlfState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                          const SvtGpuLfParams *params, int32_t dlf_avg, int32_t dlf_avg_uv,
                          int32_t temporal_layer_index, int32_t early_exit_convergence, int32_t tx_mode_only_4x4,
                          void *stream);
/* Waits for the last svtgpu_dlf_pick_async of `s` on `stream` and returns its parameters (the input parameters with
 * the picked levels; sharpness 0).  SVTGPU_ERR_INVALID_ARG: no asynchronous pick ran, or the device mode-info grid it
 * used had records out of range. */
int svtgpu_dlf_read_levels(SvtGpuDlfState *s, SvtGpuLfParams *params_out, void *stream);
/* measurement: the trial rounds the last collected asynchronous search took, and the rounds the last one enqueued
 * (a search needing more is completed by the finish kernel, one workgroup: far slower) */
int svtgpu_dlf_async_rounds(const SvtGpuDlfState *s, int32_t *taken, int32_t *enqueued);
/* A picture tiled over GPUs (svtgpu_tile_plan): the level search measures each trial's SSE over the luma
 * rectangle sse_rect = {x0, y0, x1, y1} (the rank's tile; chroma halved) and sums it over `comm` before every
 * bisection step, so every rank takes the same steps; svtgpu_dlf_frame(_to) writes only out_rect (chroma halved,
 * rounded outward), reading the input 12 samples around it.  Rect edges are multiples of 8 (or the frame edge).
 * NULL rects: the whole frame; NULL comm: no exchange. */
int svtgpu_dlf_set_tile(SvtGpuDlfState *s, const int32_t sse_rect[4], const int32_t out_rect[4], SvtGpuComm *comm);
/* LPF_PICK_FROM_Q: the loop-filter levels from the quantizer, no search (host only, no device work).
 * ≙ svt_av1_pick_filter_level_by_q (EbDeblockingFilter.c:1036-1125), the path svt_av1_pick_filter_level takes
 * for method >= LPF_PICK_FROM_Q (:1139-1146; the SB-based DLF levels 3..5).  Inputs are the fields it reads:
 * the sequence bit depth, base_q_idx, the frame / slice type, the two temporal layer indices it uses
 * (PictureControlSet's for the zero-strength threshold, the parent's for the reference-off rule), the input
 * resolution class (ResolutionRange 0..6), DlfCtrls.zero_filter_strength_lvl, the per-64x64 ME distortions
 * (rc_me_distortion, b64_count of them), and the loop-filter levels {y0, y1, u, v} of each SINGLE reference in
 * ref_frame_type_arr (compound pairs are skipped by the reference; nref = 0 for none). */
typedef struct SvtGpuDlfByQ {
    int32_t         bit_depth;                 /* 8, 10 or 12 */
    int32_t         base_q_idx;                /* 0..255 */
    int32_t         frame_type;                /* KEY_FRAME = 0 */
    int32_t         slice_type;                /* B_SLICE 0, P_SLICE 1, I_SLICE 2 */
    int32_t         temporal_layer_index;      /* pcs->temporal_layer_index */
    int32_t         ppcs_temporal_layer_index; /* pcs->ppcs->temporal_layer_index */
    int32_t         input_resolution;          /* 0..6 */
    int32_t         zero_filter_strength_lvl;  /* 0..3 */
    int32_t         b64_count;
    const uint32_t *me_sad;                    /* b64_count entries */
    int32_t         nref;                      /* 0..7 */
    int32_t         ref_levels[7][4];          /* {filter_level[0], filter_level[1], filter_level_u, filter_level_v} */
} SvtGpuDlfByQ;
int svtgpu_dlf_pick_by_q(const SvtGpuDlfByQ *in, int32_t filter_level[4]);
/* ≙ qp_based_dlf_param (EbDeblockingFilter.c:992-1031): luma / chroma level guesses from base_q_idx */
int svtgpu_dlf_qp_based_param(int32_t bit_depth, int32_t base_q_idx, int32_t frame_type, int32_t *filter_level_y,
                              int32_t *filter_level_uv);

/* Σ (a - b)^2 over one plane (svt_spatial_full_distortion_kernel / svt_full_distortion_kernel16_bits
 * over the frame, EbDeblockingFilter.c:716-838). Synchronous. */
int svtgpu_plane_sse(const SvtGpuFrame *a, const SvtGpuFrame *b, int32_t plane, uint64_t *sse, void *stream);


/* =========================================================================================
 * Mode-decision distortion: SAD / SSE / variance
 * ========================================================================================= */
/* RTCD-compatible per-block shims, one per AV1 block size (BlockSize order).  Synchronous.
 *   svtgpu_aom_sad{W}x{H}              ≙ svt_aom_sad{W}x{H}            (aom_dsp_rtcd.h:264-350, C EbComputeSAD_C.c:117-206)
 *   svtgpu_aom_sad{W}x{H}x4d           ≙ svt_aom_sad{W}x{H}x4d
 *   svtgpu_aom_variance{W}x{H}         ≙ svt_aom_variance{W}x{H}       (aom_dsp_rtcd.h:480-540, C variance.c:300-345)
 *   svtgpu_aom_highbd_10_variance{W}x{H} ≙ svt_aom_highbd_10_variance{W}x{H} (aom_dsp_rtcd.h:544-570, C EbPsnr.c:174-214);
 *       its pointers are CONVERT_TO_BYTEPTR-encoded uint16_t planes, as in the reference (EbDefinitions.h:950-951). */
uint32_t     svtgpu_aom_sad4x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad4x4x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance4x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance4x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad4x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad4x8x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance4x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance4x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad8x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad8x4x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance8x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance8x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad8x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad8x8x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance8x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance8x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad8x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad8x16x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance8x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance8x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad16x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad16x8x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance16x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance16x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad16x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad16x16x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance16x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance16x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad16x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad16x32x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance16x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance16x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad32x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad32x16x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance32x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance32x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad32x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad32x32x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance32x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance32x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad32x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad32x64x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance32x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance32x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad64x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad64x32x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance64x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance64x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad64x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad64x64x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance64x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance64x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad64x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad64x128x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance64x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance64x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad128x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad128x64x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance128x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance128x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad128x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad128x128x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance128x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance128x128(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad4x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad4x16x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance4x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance4x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad16x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad16x4x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance16x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance16x4(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad8x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad8x32x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance8x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance8x32(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad32x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad32x8x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance32x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance32x8(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad16x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad16x64x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance16x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance16x64(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
uint32_t     svtgpu_aom_sad64x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride);
void         svtgpu_aom_sad64x16x4d(const uint8_t *src, int src_stride, const uint8_t *const ref[], int ref_stride, uint32_t *sad_array);
unsigned int svtgpu_aom_variance64x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
unsigned int svtgpu_aom_highbd_10_variance64x16(const uint8_t *src, int src_stride, const uint8_t *ref, int ref_stride, unsigned int *sse);
/* ≙ sad_16b_kernel (aom_dsp_rtcd.h:861, C svt_aom_sad_16b_kernel_c EbComputeSAD_C.c:39) */
uint32_t svtgpu_sad_16b_kernel(uint16_t *src, uint32_t src_stride, uint16_t *ref, uint32_t ref_stride, uint32_t height,
                               uint32_t width);
/* ≙ svt_aom_sse / svt_aom_highbd_sse (aom_dsp_rtcd.h:54-56, C EbEncInterPrediction.c:562-590; highbd takes plain
 * uint16_t planes cast to uint8_t*) */
int64_t svtgpu_aom_sse(const uint8_t *a, int a_stride, const uint8_t *b, int b_stride, int width, int height);
int64_t svtgpu_aom_highbd_sse(const uint8_t *a8, int a_stride, const uint8_t *b8, int b_stride, int width, int height);
/* ≙ svt_spatial_full_distortion_kernel / svt_full_distortion_kernel16_bits (common_dsp_rtcd.h:169-171) */
uint64_t svtgpu_spatial_full_distortion_kernel(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                               uint8_t *recon, int32_t recon_offset, uint32_t recon_stride,
                                               uint32_t area_width, uint32_t area_height);
uint64_t svtgpu_full_distortion_kernel16_bits(uint8_t *input, uint32_t input_offset, uint32_t input_stride,
                                              uint8_t *recon, int32_t recon_offset, uint32_t recon_stride,
                                              uint32_t area_width, uint32_t area_height);
/* ≙ svt_nxm_sad_kernel / svt_nxm_sad_kernel_sub_sampled (aom_dsp_rtcd.h:853-854): the MD fast-loop N x M SAD
 * (C svt_fast_loop_nxm_sad_kernel, EbComputeSAD_C.c:20; the C "sub-sampled" entry is the full SAD too, :209) */
uint32_t svtgpu_nxm_sad_kernel(const uint8_t *src, uint32_t src_stride, const uint8_t *ref, uint32_t ref_stride,
                               uint32_t height, uint32_t width);
uint32_t svtgpu_nxm_sad_kernel_sub_sampled(const uint8_t *src, uint32_t src_stride, const uint8_t *ref,
                                           uint32_t ref_stride, uint32_t height, uint32_t width);
/* ≙ svt_aom_mse16x16 (aom_dsp_rtcd.h:241, C EbPsnr.c:76) and svt_aom_highbd_8_mse16x16 (:262, C variance.c:453;
 * 16-bit samples CONVERT_TO_BYTEPTR-encoded, *sse only) */
uint32_t svtgpu_aom_mse16x16(const uint8_t *src_ptr, int32_t source_stride, const uint8_t *ref_ptr,
                             int32_t recon_stride, uint32_t *sse);
void     svtgpu_aom_highbd_8_mse16x16(const uint8_t *src_ptr, int32_t source_stride, const uint8_t *ref_ptr,
                                      int32_t recon_stride, uint32_t *sse);
/* ≙ variance_highbd (aom_dsp_rtcd.h:867, C svt_aom_variance_highbd_c variance.c:278): any w x h, 16-bit */
uint32_t svtgpu_aom_variance_highbd(const uint16_t *a, int a_stride, const uint16_t *b, int b_stride, int w, int h,
                                    uint32_t *sse);
/* ≙ svt_aom_sub_pixel_variance{W}x{H} (aom_dsp_rtcd.h:587-753, C SUBPIX_VAR variance.c:308): 2-tap bilinear
 * (1/8 pel offsets xoffset, yoffset in 0..7) of a (H + 1) x (W + 1) source window, then the W x H variance */
uint32_t svtgpu_aom_sub_pixel_variance4x4(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance4x8(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance8x4(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance8x8(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance8x16(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance16x8(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance16x16(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance16x32(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance32x16(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance32x32(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance32x64(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance64x32(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance64x64(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance64x128(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance128x64(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance128x128(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance4x16(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance16x4(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance8x32(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance32x8(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance16x64(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);
uint32_t svtgpu_aom_sub_pixel_variance64x16(const uint8_t *src_ptr, int source_stride, int xoffset, int yoffset, const uint8_t *ref_ptr, int ref_stride, uint32_t *sse);

/* Batched MD distortion (the frame-level GPU boundary; no single reference equivalent: it evaluates what
 * the MD candidate loops evaluate block by block through svt_aom_mefn_ptr, av1me.c:29-174).
 * For every 64x64 SB of `source` and every reference frame r at the SB's full-pel motion vector
 * mv[sb][r] = {x, y}, svtgpu_md_dist_batch computes the raw moments of every 4x4 cell of the SB (moments[sb][r][256],
 * cells in raster order, 8 bytes each: x = SAD | (uint16_t)(signed sum) << 16, y = SSE of the differences): every
 * block of every AV1 shape <= 64x64 tiling the SB has exact sums of its cells' moments.  svtgpu_md_expand derives,
 * for an SB range, every block's
 *   q = 0: SAD (sad{W}x{H} / sad_16b_kernel), q = 1: the *sse the variance function reports,
 *   q = 2: the variance (8-bit: svt_aom_variance{W}x{H}; 10-bit: svt_aom_highbd_10_variance{W}x{H}, which round only
 *          the block totals, EbPsnr.c:183-214);
 * svtgpu_md_read expands and reads an SB range.
 * Samples outside the frame read the nearest edge sample (the encoder's padded pictures).
 * Expanded layout: out[sb][r][q][SVTGPU_MD_BLOCKS]; shapes in BlockSize order without the 128 shapes,
 * blocks of one shape in raster order (svtgpu_md_layout). */
#define SVTGPU_MD_SHAPES 19
#define SVTGPU_MD_BLOCKS 849
typedef struct SvtGpuMdBatch SvtGpuMdBatch;
int     svtgpu_md_batch_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t nref, SvtGpuMdBatch **out);
void    svtgpu_md_batch_destroy(SvtGpuMdBatch *b);
int32_t svtgpu_md_batch_nsb(const SvtGpuMdBatch *b);
int     svtgpu_md_set_mvs(SvtGpuMdBatch *b, const int16_t *mv, void *stream); /* host [nsb][nref][2] */
int     svtgpu_md_dist_batch(SvtGpuMdBatch *b, const SvtGpuFrame *source, const SvtGpuFrame *const *refs,
                             int32_t sb_begin, int32_t sb_end, void *stream);
/* every block's values of SBs [sb_begin, sb_end) from the last batch's moments, into the expanded table (in stream
 * order; svtgpu_md_out_device_ptr) -- for a consumer that wants per-shape values rather than the moments */
int     svtgpu_md_expand(SvtGpuMdBatch *b, int32_t sb_begin, int32_t sb_end, void *stream);
/* expands SBs [sb_begin, sb_end) and copies their rows [sb][r][3][SVTGPU_MD_BLOCKS] to `out` (synchronous) */
int     svtgpu_md_read(SvtGpuMdBatch *b, uint32_t *out, int32_t sb_begin, int32_t sb_end, void *stream);
void   *svtgpu_md_out_device_ptr(SvtGpuMdBatch *b);     /* the expanded table [nsb][nref][3][SVTGPU_MD_BLOCKS] */
void   *svtgpu_md_moments_device_ptr(SvtGpuMdBatch *b); /* the cell moments [nsb][nref][256] (uint32 pairs) */
/* shape_w/shape_h/shape_offset: [SVTGPU_MD_SHAPES] block dims and first output index of each shape */
void    svtgpu_md_layout(int32_t *shape_w, int32_t *shape_h, int32_t *shape_offset);


/* =========================================================================================
 * Open-loop motion-estimation SAD
 * ========================================================================================= */
#ifndef SVTGPU_BOOL_T
#define SVTGPU_BOOL_T
typedef uint8_t Bool; /* EbSvtAv1.h:82 */
#endif
/* RTCD-compatible shims (synchronous, host pointers), each replacing the pointer it names:
 * svt_ext_all_sad_calculation_8x8_16x16 (aom_dsp_rtcd.h:850; C EbMotionEstimation.c:336) -- 8 positions x .. x+7 of a
 *   64x64 block: 8x8 / 16x16 SADs (Z-order), best SAD/MV updates (strict <), p_eight_sad16x16[16][8] */
void svtgpu_ext_all_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                              uint32_t mv, uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16,
                                              uint32_t *p_best_mv8x8, uint32_t *p_best_mv16x16,
                                              uint32_t p_eight_sad16x16[16][8], uint32_t p_eight_sad8x8[64][8],
                                              Bool sub_sad);
/* svt_ext_eight_sad_calculation_32x32_64x64 (aom_dsp_rtcd.h:851; C EbMotionEstimation.c:370) */
void svtgpu_ext_eight_sad_calculation_32x32_64x64(uint32_t p_sad16x16[16][8], uint32_t *p_best_sad_32x32,
                                                  uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                                  uint32_t *p_best_mv64x64, uint32_t mv, uint32_t p_sad32x32[4][8]);
/* svt_ext_sad_calculation_8x8_16x16 (aom_dsp_rtcd.h:839; C EbMotionEstimation.c:99) -- one 16x16 at one position */
void svtgpu_ext_sad_calculation_8x8_16x16(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                                          uint32_t *p_best_sad_8x8, uint32_t *p_best_sad_16x16, uint32_t *p_best_mv8x8,
                                          uint32_t *p_best_mv16x16, uint32_t mv, uint32_t *p_sad16x16,
                                          uint32_t *p_sad8x8, Bool sub_sad);
/* svt_ext_sad_calculation_32x32_64x64 (aom_dsp_rtcd.h:845; C EbMotionEstimation.c:172) */
void svtgpu_ext_sad_calculation_32x32_64x64(uint32_t *p_sad16x16, uint32_t *p_best_sad_32x32,
                                            uint32_t *p_best_sad_64x64, uint32_t *p_best_mv32x32,
                                            uint32_t *p_best_mv64x64, uint32_t mv, uint32_t *p_sad32x32);
/* svt_sad_loop_kernel (aom_dsp_rtcd.h:776; C EbComputeSAD_C.c:58) -- full search of a block over an area */
void svtgpu_sad_loop_kernel(uint8_t *src, uint32_t src_stride, uint8_t *ref, uint32_t ref_stride,
                            uint32_t block_height, uint32_t block_width, uint64_t *best_sad, int16_t *x_search_center,
                            int16_t *y_search_center, uint32_t src_stride_raw, uint8_t skip_search_line,
                            int16_t search_area_width, int16_t search_area_height);
/* svt_pme_sad_loop_kernel (aom_dsp_rtcd.h:866; C EbProductCodingLoop.c:1801) -- the MD full-pel refinement: cost =
 * SAD + svt_aom_fp_mv_err_cost (mcomp.c:771) over the reference's visiting order; mv_cost_params is the reference's
 * MV_COST_PARAMS (mcomp.h:37), read with its layout */
struct svt_mv_cost_param;
void svtgpu_pme_sad_loop_kernel(const struct svt_mv_cost_param *mv_cost_params, uint8_t *src, uint32_t src_stride,
                                uint8_t *ref, uint32_t ref_stride, uint32_t block_height, uint32_t block_width,
                                uint32_t *best_cost, int16_t *best_mvx, int16_t *best_mvy,
                                int16_t search_position_start_x, int16_t search_position_start_y,
                                int16_t search_area_width, int16_t search_area_height, int16_t search_step,
                                int16_t mvx, int16_t mvy);
/* Frame level: the integer full-pel search of every 64x64 block against every reference (≙ the per-block
 * open_loop_me_fullpel_search_sblock, EbMotionEstimation.c:782-818, after the best SADs are reset to MAX_SAD_VALUE,
 * :1363-1364).  origin[sb][r] = {x, y} is the search-area origin relative to the block (the MV of search position
 * (0, 0)); the search covers sa_w x sa_h positions (sa_w <= 192); sub_sad = the SUB_SAD_SEARCH method (8x8 SADs over
 * rows 0, 2, 4, 6, doubled).  8-bit luma; reference samples outside the frame read the nearest edge sample (the
 * padded reference pictures).  Output per (sb, r): 85 best SADs and MVs -- [0, 64) 8x8, [64, 80) 16x16, [80, 84) 32x32,
 * [84] 64x64, in the reference's Z-order numbering (me_ctx->p_best_sad_8x8 ...); MV = (y << 16) | (uint16_t)x. */
#define SVTGPU_ME_BLOCKS 85
typedef struct SvtGpuMeBatch SvtGpuMeBatch;
int  svtgpu_me_batch_create(SvtGpuContext *ctx, int32_t width, int32_t height, int32_t nref, SvtGpuMeBatch **out);
void svtgpu_me_batch_destroy(SvtGpuMeBatch *b);
int  svtgpu_me_set_origins(SvtGpuMeBatch *b, const int16_t *origin, void *stream); /* host [nsb][nref][2] */
int  svtgpu_me_search(SvtGpuMeBatch *b, const SvtGpuFrame *source, const SvtGpuFrame *const *refs, int32_t sa_w,
                      int32_t sa_h, int32_t sub_sad, int32_t sb_begin, int32_t sb_end, void *stream);
int  svtgpu_me_read(SvtGpuMeBatch *b, uint32_t *best_sad, uint32_t *best_mv, int32_t sb_begin, int32_t sb_end,
                    void *stream); /* host [sb_end - sb_begin][nref][85] each (nullable) */

/* =========================================================================================
 * Frame-buffer work around the path
 * ========================================================================================= */
/* RTCD-compatible shims (synchronous, host pointers):
 * svt_convert_8bit_to_16bit / svt_convert_16bit_to_8bit (common_dsp_rtcd.h:154-156; C EbPackUnPack_C.c:270-283) */
void svtgpu_convert_8bit_to_16bit(uint8_t *src, uint32_t src_stride, uint16_t *dst, uint32_t dst_stride, uint32_t width,
                                  uint32_t height);
void svtgpu_convert_16bit_to_8bit(uint16_t *src, uint32_t src_stride, uint8_t *dst, uint32_t dst_stride, uint32_t width,
                                  uint32_t height);
/* svt_aom_generate_padding / svt_aom_generate_padding16_bit (EbMcp.h:46-51; C EbMcp.c:95-240): src_pic is the padded
 * buffer's first sample, the visible area starts at (padding_width, padding_height) */
void svtgpu_aom_generate_padding(uint8_t *src_pic, uint32_t src_stride, uint32_t original_src_width,
                                 uint32_t original_src_height, uint32_t padding_width, uint32_t padding_height);
void svtgpu_aom_generate_padding16_bit(uint16_t *src_pic, uint32_t src_stride, uint32_t original_src_width,
                                       uint32_t original_src_height, uint32_t padding_width, uint32_t padding_height);
/* svt_extend_frame (EbRestoration.c:197): data = first visible sample (CONVERT_TO_BYTEPTR-encoded when highbd) */
void svtgpu_extend_frame(uint8_t *data, int32_t width, int32_t height, int32_t stride, int32_t border_horz,
                         int32_t border_vert, int32_t highbd);
/* Device-pointer versions (asynchronous on `stream`, nullable = the library's default stream); bits = 8 or 16,
 * strides in samples: */
int svtgpu_convert_plane(const void *src, int32_t src_bits, int32_t src_stride, void *dst, int32_t dst_bits,
                         int32_t dst_stride, int32_t width, int32_t height, void *stream);
int svtgpu_pad_plane(void *buf, int32_t bits, int32_t stride, int32_t width, int32_t height, int32_t pad_width,
                     int32_t pad_height, void *stream);
int svtgpu_extend_plane(void *data, int32_t bits, int32_t stride, int32_t width, int32_t height, int32_t border_horz,
                        int32_t border_vert, void *stream);
/* svt_convert_pic_8bit_to_16bit (EbRestProcess.c:235-272) and the 16 -> 8 copy-back of non-reference pictures
 * (EbRestProcess.c:670-697) on device frames: all three planes, direction from the frames' bit depths */
int svtgpu_frame_convert(const SvtGpuFrame *src, SvtGpuFrame *dst, void *stream);

/* =========================================================================================
 * Loop restoration
 * ========================================================================================= */
/* RTCD-compatible per-block shims (common_dsp_rtcd.h:174-185).  The Wiener convolve reads round_0 / round_1 of
 * the ConvolveParams (full layout at the top of this header); 16-bit planes are passed CONVERT_TO_BYTEPTR-encoded
 * (EbDefinitions.h:950-951), as in the reference. */
/* ≙ svt_av1_wiener_convolve_add_src (C convolve.c:109-151): 8-tap separable, src row/col -3..+4 */
void svtgpu_av1_wiener_convolve_add_src(const uint8_t *src, ptrdiff_t src_stride, uint8_t *dst, ptrdiff_t dst_stride,
                                        const int16_t *filter_x, const int16_t *filter_y, int32_t w, int32_t h,
                                        const SVTGPU_CONVOLVE_PARAMS_T *conv_params);
/* ≙ svt_av1_highbd_wiener_convolve_add_src (C convolve.c:194-232) */
void svtgpu_av1_highbd_wiener_convolve_add_src(const uint8_t *src, ptrdiff_t src_stride, uint8_t *dst,
                                               ptrdiff_t dst_stride, const int16_t *filter_x,
                                               const int16_t *filter_y, int32_t w, int32_t h,
                                               const SVTGPU_CONVOLVE_PARAMS_T *conv_params, int32_t bd);
/* ≙ svt_av1_selfguided_restoration (C EbRestoration.c:923-955): flt0/flt1 of one processing unit, input read
 * with a 3-sample border */
void svtgpu_av1_selfguided_restoration(const uint8_t *dgd8, int32_t width, int32_t height, int32_t dgd_stride,
                                       int32_t *flt0, int32_t *flt1, int32_t flt_stride, int32_t sgr_params_idx,
                                       int32_t bit_depth, int32_t highbd);
/* ≙ svt_apply_selfguided_restoration (C EbRestoration.c:957-991) */
void svtgpu_apply_selfguided_restoration(const uint8_t *dat8, int32_t width, int32_t height, int32_t stride,
                                         int32_t eps, const int32_t *xqd, uint8_t *dst8, int32_t dst_stride,
                                         int32_t *tmpbuf, int32_t bit_depth, int32_t highbd);
/* ≙ svt_av1_compute_stats / _highbd (aom_dsp_rtcd.h:66-68, C EbRestorationPick.c:671 / :708): the Wiener
 * statistics M[win^2] and H[win^2][win^2] of a unit; dgd read with a win/2 border */
void svtgpu_av1_compute_stats(int32_t wiener_win, const uint8_t *dgd8, const uint8_t *src8, int32_t h_start,
                              int32_t h_end, int32_t v_start, int32_t v_end, int32_t dgd_stride, int32_t src_stride,
                              int64_t *M, int64_t *H);
void svtgpu_av1_compute_stats_highbd(int32_t wiener_win, const uint8_t *dgd8, const uint8_t *src8, int32_t h_start,
                                     int32_t h_end, int32_t v_start, int32_t v_end, int32_t dgd_stride,
                                     int32_t src_stride, int64_t *M, int64_t *H, SVTGPU_BIT_DEPTH_T bit_depth);
/* ≙ svt_av1_lowbd_pixel_proj_error / svt_av1_highbd_pixel_proj_error (aom_dsp_rtcd.h:79-81, C :167 / :232) */
int64_t svtgpu_av1_lowbd_pixel_proj_error(const uint8_t *src8, int32_t width, int32_t height, int32_t src_stride,
                                          const uint8_t *dat8, int32_t dat_stride, int32_t *flt0, int32_t flt0_stride,
                                          int32_t *flt1, int32_t flt1_stride, int32_t xq[2],
                                          const SVTGPU_SGR_PARAMS_T *params);
int64_t svtgpu_av1_highbd_pixel_proj_error(const uint8_t *src8, int32_t width, int32_t height, int32_t src_stride,
                                           const uint8_t *dat8, int32_t dat_stride, int32_t *flt0, int32_t flt0_stride,
                                           int32_t *flt1, int32_t flt1_stride, int32_t xq[2],
                                           const SVTGPU_SGR_PARAMS_T *params);
/* ≙ svt_get_proj_subspace (aom_dsp_rtcd.h:212, C EbRestorationPick.c:560): least-squares xq of a unit */
void svtgpu_get_proj_subspace(const uint8_t *src8, int width, int height, int src_stride, const uint8_t *dat8,
                              int dat_stride, int use_highbitdepth, int32_t *flt0, int flt0_stride, int32_t *flt1,
                              int flt1_stride, int *xq, const SVTGPU_SGR_PARAMS_T *params);

/* Per restoration unit parameters (RestorationUnitInfo, EbRestoration.h:169-188). */
#define SVTGPU_RESTORE_NONE 0
#define SVTGPU_RESTORE_WIENER 1
#define SVTGPU_RESTORE_SGRPROJ 2
typedef struct SvtGpuRestUnit {
    int32_t type;       /* SVTGPU_RESTORE_* */
    int16_t vfilter[8]; /* WienerInfo */
    int16_t hfilter[8];
    int32_t ep;         /* SgrprojInfo */
    int32_t xqd[2];
} SvtGpuRestUnit;

typedef struct SvtGpuLrState SvtGpuLrState;
/* unit_size[plane]: restoration_unit_size (64/128/256 luma; chroma usually luma >> 1).  width / height: the
 * picture's crop size (frm_size.frame_width / _height, EbPictureControlSet.c:1207; any size >= 8), which the
 * restoration units, the search and the filter cover (chroma (width + 1) >> 1, the reference's crop_widths); the
 * frames handed to the search and the apply are the 8-aligned coded size (the deblocking / CDEF extent, mi_cols x 4).
 * Samples right of / below the crop keep the CDEF output in the apply. */
int  svtgpu_lr_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, const int32_t unit_size[3],
                            SvtGpuLrState **out);
void svtgpu_lr_state_destroy(SvtGpuLrState *s);
/* number of units of a plane: horz/vert units (count_units_in_tile, EbRestoration.c:122-124) */
int  svtgpu_lr_units(const SvtGpuLrState *s, int32_t plane, int32_t *hunits, int32_t *vunits);
int  svtgpu_lr_set_units(SvtGpuLrState *s, int32_t plane, const SvtGpuRestUnit *units, void *stream);
/* ≙ svt_av1_loop_restoration_filter_frame(rst_tmpbuf, frame, cm, 0) (EbRestoration.c:1179-1255) with the
 * stripe boundary lines of svt_av1_loop_restoration_save_boundary_lines (EbRestoration.c:1682): rows above /
 * below each 64-row processing stripe come from `deblocked` (the DLF output) inside the frame and from
 * `cdef_out` at the frame top/bottom.  Writes every sample of `out` (planes whose frame_type is NONE are
 * copied).  frame_type[plane]: SVTGPU_RESTORE_NONE or any other value (= per-unit types apply); frame_type == NULL:
 * every plane unit by unit with the units the last search left on the device (svtgpu_lr_search_frame_async: a plane
 * whose frame type came out NONE holds NONE units, which are copied) -- no host round trip between search and apply. */
int  svtgpu_lr_apply_frame(SvtGpuLrState *s, const SvtGpuFrame *deblocked, const SvtGpuFrame *cdef_out,
                           SvtGpuFrame *out, const int32_t frame_type[3], void *stream);


/* Loop-restoration search controls (WnFilterCtrls / SgFilterCtrls, EncModeConfig.c:1329-1445, fixed-range SGR
 * search: step_range 16) and the encoder's rate inputs (Macroblock rdmult / restore costs). */
typedef struct SvtGpuLrSearchControls {
    int32_t wn_enabled, wn_use_chroma, wn_filter_tap_lvl, wn_use_refinement, wn_max_one_refinement_step;
    int32_t sg_enabled, sg_use_chroma;
    int32_t sg_start_ep[2], sg_end_ep[2], sg_ep_inc[2], sg_refine[2]; /* [luma, chroma] */
    int32_t rdmult;
    int32_t switchable_restore_cost[3], wiener_restore_cost[2], sgrproj_restore_cost[2];
} SvtGpuLrSearchControls;
/* Per-unit search record (RestUnitSearchInfo, EbRestoration.h:349-360). */
typedef struct SvtGpuLrUnitSearch {
    int64_t        sse[3];        /* NONE, WIENER (INT64_MAX = no filter), SGRPROJ */
    SvtGpuRestUnit wiener, sgrproj; /* best parameters of each type */
} SvtGpuLrUnitSearch;
/* ≙ restoration_seg_search over every segment + rest_finish_search (EbRestorationPick.c:1471-1634) on the CDEF
 * output `recon` against `source`; sets the units of `s` (frame types in frame_type_out[3]) and, if
 * search_out[plane] is non-NULL, returns the per-unit records.  Synchronous. */
int svtgpu_lr_search_frame(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                           const SvtGpuLrSearchControls *ctrls, int32_t frame_type_out[3],
                           SvtGpuLrUnitSearch *const search_out[3], void *stream);
/* The asynchronous form of svtgpu_lr_search_frame (≙ restoration_seg_search + rest_finish_search with no host wait):
 * the search, the per-unit records and the RD finish (rest_finish_search, EbRestorationPick.c:1555-1634) are enqueued
 * on `stream` and set the state's units in stream order; a picture tiled over GPUs sums the records over its
 * communicator on the device first.  Returns without waiting.  svtgpu_lr_apply_frame(..., frame_type = NULL, ...)
 * applies the result in stream order; svtgpu_lr_read_result waits for it and returns the frame types (and a failure
 * of the device search, e.g. a descent's bound, which this call cannot see).  SVTGPU_LR_FINISH=host: the round-5 form
 * (the records read back, the finish on the host, one wait inside this call). */
int svtgpu_lr_search_frame_async(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                                 const SvtGpuLrSearchControls *ctrls, void *stream);
/* Waits for the last asynchronous search of `s` queued on `stream` and returns its frame types (SVTGPU_RESTORE_*);
 * after a synchronous search, or a second call, the last frame types collected.  SVTGPU_ERR_HIP: the device search
 * failed (svtgpu_error_string names it). */
int svtgpu_lr_read_result(SvtGpuLrState *s, int32_t frame_type_out[3], void *stream);
/* The state's units of one plane (the RestorationUnitInfo the frame header / tile coding writes: the last search's
 * picks, NONE units for a plane whose frame type is NONE); waits for an asynchronous search first. */
int svtgpu_lr_read_units(SvtGpuLrState *s, int32_t plane, SvtGpuRestUnit *units_out, void *stream);
/* Per-unit part of the search for a band of unit rows: the units of unit rows [row_begin[p], row_end[p]) of each
 * searched plane (restoration_seg_search restricted to those units; every unit's search is independent of the
 * others).  Writes those units' records into search_out[p] (arrays of all units of the plane, row-major; other
 * entries untouched); no RD finish and the state's units are not changed.  The multi-GPU split of the search:
 * every rank searches a band, the records are gathered and svtgpu_lr_finish_plane picks on every rank.
 * Synchronous. */
int svtgpu_lr_search_units(SvtGpuLrState *s, const SvtGpuFrame *recon, const SvtGpuFrame *source,
                           const SvtGpuLrSearchControls *ctrls, const int32_t row_begin[3], const int32_t row_end[3],
                           SvtGpuLrUnitSearch *const search_out[3], void *stream);
/* ≙ rest_finish_search of one plane (EbRestorationPick.c:1555-1634): the frame restoration type and the units'
 * types/parameters (copy_unit_info) from the records of all `nunits` units of the plane.  Host only (no device
 * work, usable without a GPU); returns SVTGPU_OK with *frame_type_out = NONE for a plane that is not searched. */
int svtgpu_lr_finish_plane(const SvtGpuLrSearchControls *ctrls, int32_t plane, int32_t nunits,
                           const SvtGpuLrUnitSearch *records, int32_t *frame_type_out, SvtGpuRestUnit *units_out);
/* ≙ rest_finish_search of the whole frame (EbRestorationPick.c:1555-1634): the planes in order over one
 * RestUnitSearchInfo array shared by the planes, as the reference allocates it -- a chroma plane's switchable pass reads
 * luma's entries for a filter type chroma does not search (Wiener level 5 beside self-guided level 1-3: presets 3-9),
 * which svtgpu_lr_finish_plane on one plane alone cannot.  nunits[p] / records[p] / units_out[p] for the searched
 * planes (units_out of the others zeroed when non-NULL).  Host only. */
int svtgpu_lr_finish_frame(const SvtGpuLrSearchControls *ctrls, const int32_t nunits[3],
                           const SvtGpuLrUnitSearch *const records[3], int32_t frame_type_out[3],
                           SvtGpuRestUnit *const units_out[3]);
/* A picture tiled over GPUs (svtgpu_tile_plan): svtgpu_lr_search_frame searches only the units of units[p] = {col0,
 * row0, col1, row1} of each plane, sums the zero-padded per-unit records over `comm` (the gather), and runs the RD
 * finish of every plane on every rank (the same frame types and units everywhere); svtgpu_lr_apply_frame writes only
 * out[p] = {x0, y0, x1, y1} (plane samples), reading the CDEF output 3 samples and the DLF output 3 rows around it.
 * NULL arrays: the whole frame; NULL comm: no exchange. */
int svtgpu_lr_set_tile(SvtGpuLrState *s, const int32_t units[3][4], const int32_t out[3][4], SvtGpuComm *comm);
/* Device-time profile of the searches timed since the previous read, by kernel class: 0 unit sums + Wiener
 * statistics, 1 self-guided filters (sgr_flt_kernel), 2 Wiener descents (wiener_res_kernel), 3 self-guided searches
 * (sgr_res_kernel: moments, seeds and descents), 4 Wiener decomposition and the chosen ep's SSE, 5 unused.  Each
 * launch is timed from its first workgroup's start to its last workgroup's end on the device's 100 MHz
 * s_memrealtime clock (per-launch HIP event packets would cost more than these launches); bytes = algorithmic
 * HBM bytes of the class (compulsory reads/writes of the samples and filter planes the launches touch). */
typedef struct SvtGpuLrProfile {
    int32_t launches[6]; /* totals over `searches` searches */
    float   ms[6];        /* the device clock: first workgroup start to last workgroup end of each launch */
    double  bytes[6];
    int32_t searches;
    float   ms_events[6]; /* HIP events around each launch on its stream (the span rocprofv3's kernel trace reports) */
} SvtGpuLrProfile;
/* enable != 0 turns timing of the following searches on (0 off): a bit mask of the classes to time (bit c =
 * class c; -1 = all); bit 6 also brackets each timed launch with HIP events (ms_events: the span rocprofv3 reports;
 * events between launches can change how the two LR chains interleave, so they are a separate, opt-in bit); bit 7 runs
 * the Wiener chain on the caller's stream after the self-guided one instead of beside it, so every search kernel has the
 * device to itself and its duration is its own (measurement only: slower searches).  `totals` (nullable) first receives the sums over the searches timed since the previous read
 * (untimed classes read 0), which are then reset; reading synchronizes the device.  The timings accumulate on the
 * device: a timed search adds one small launch and no copies or host synchronization. */
int svtgpu_lr_profile(SvtGpuLrState *s, int32_t enable, SvtGpuLrProfile *totals);
/* Host <-> device bytes moved by the frame-level entry points since the last reset (copies and the results read from
 * mapped memory; per-block shims excluded) -- measurement only, no reference counterpart.  reset != 0 zeroes them. */
int svtgpu_transfer_bytes(uint64_t *h2d, uint64_t *d2h, int32_t reset);
/* controls of wn_filter_lvl / sg_filter_lvl (EncModeConfig.c:1329-1445); rate fields are left zero */
int svtgpu_lr_controls_for_level(int32_t wn_level, int32_t sg_level, SvtGpuLrSearchControls *c);

/* ---------------------------------------------------------------------------------------------
 * CCSO, cross-component sample offset: the fork's AVM experiment, EbCcso.c / EbPickccso.c.
 * The fork's encoder never calls it (EbCdefProcess.c:621-623 comment the search and the apply out); these entry points
 * are what an encoder that re-enables it binds.  Geometry as the reference's: every plane's samples are addressed with
 * the luma width as stride (ccso_stride, EbPickccso.c:800), chroma planes are (width >> 1) x (height >> 1) (the
 * unpadded size >> 1, svt_av1_setup_dst_planes, EbDeblockingFilter.c:114-116), the classifier reads the luma plane
 * padded by SVTGPU_CCSO_PAD samples (ext_rec_y, stride width + 2 * SVTGPU_CCSO_PAD), and the filter blocks are
 * 256 x 256 luma / 128 x 128 chroma samples (CCSO_BLK_SIZE 7, EbDefinitions.h:1409), counted on the 8-aligned mode-info
 * grid: nvfb x nhfb (derive_ccso_filter, EbPickccso.c:473-476).
 * --------------------------------------------------------------------------------------------- */
#define SVTGPU_CCSO_PAD 5     /* CCSO_PADDING_SIZE (EbDefinitions.h:1410) */
#define SVTGPU_CCSO_LUT 2048  /* CCSO_BAND_NUM * 16 (EbDefinitions.h:1411) */
/* one plane of FrameHeader.ccso_info (EbAv1Structs.h:407-427); filter_offset index (band << 4) + (cls0 << 2) + cls1 */
typedef struct SvtGpuCcsoParams {
    uint8_t enable, bo_only, quant_idx, ext_filter_support, max_band_log2, edge_clf, reserved[2];
    int8_t  filter_offset[SVTGPU_CCSO_LUT];
} SvtGpuCcsoParams;
/* the filter-block grid of a plane (nvfb rows x nhfb columns; the block flags arrays are nvfb * nhfb bytes, row-major) */
int svtgpu_ccso_grid(int32_t width, int32_t height, int32_t plane, int32_t *nvfb, int32_t *nhfb);
/* ≙ the ext_rec_y construction (the copy of EbPickccso.c:907-918 + extend_ccso_border, EbCcso.c:185-201): the luma
 * plane (8- or 16-bit samples, device) into `ext` (device, (height + 10) rows of width + 10 uint16), replicated
 * SVTGPU_CCSO_PAD samples on every side. */
int svtgpu_ccso_extend_luma(const void *luma, int32_t bits, int32_t stride, int32_t width, int32_t height,
                            uint16_t *ext, void *stream);
typedef struct SvtGpuCcsoState SvtGpuCcsoState;
int  svtgpu_ccso_state_create(SvtGpuContext *ctx, int32_t width, int32_t height, SvtGpuCcsoState **out);
void svtgpu_ccso_state_destroy(SvtGpuCcsoState *s);
/* ≙ derive_ccso_filter (EbPickccso.c:464-779) of one plane: every (band-offset-only, filter support, quantization step,
 * edge classifier, band count) configuration trained as the reference trains it, the cheapest kept, then weighed
 * against the unfiltered plane.  ext (device, svtgpu_ccso_extend_luma of the pre-filter luma), org / rec (device,
 * uint16, stride = width).  rdmult as derive_ccso_filter receives it (ccso_search's weighting applied).  Results stay
 * in the state for svtgpu_ccso_apply_plane(..., params = NULL); params_out / flags_out (host, nullable) also receive
 * them (one wait).  A disabled plane reads enable = 0 and zero fields / flags. */
int svtgpu_ccso_search_plane(SvtGpuCcsoState *s, const uint16_t *ext, const uint16_t *org, const uint16_t *rec,
                             int32_t plane, int32_t bit_depth, int32_t rdmult, SvtGpuCcsoParams *params_out,
                             uint8_t *flags_out, void *stream);
/* ≙ ccso_search (EbPickccso.c:785-815): rdmult weighted by clamp(base_q_idx, 1, 63), the three planes searched side by
 * side (one launch per pass).  Returns 1 and searches nothing when the weighted rdmult reaches INT_MAX (the reference
 * returns early); *frame_flag = ccso_frame_flag (any plane enabled).  params_out = NULL: nothing is read back and
 * nothing waited for (*frame_flag = 0); the results stay in the state for svtgpu_ccso_apply_plane(..., NULL, ...). */
int svtgpu_ccso_search_frame(SvtGpuCcsoState *s, const uint16_t *ext, const uint16_t *const org[3],
                             const uint16_t *const rec[3], int32_t bit_depth, int32_t rdmult, int32_t base_q_idx,
                             SvtGpuCcsoParams params_out[3], uint8_t *const flags_out[3], int32_t *frame_flag,
                             void *stream);
/* ≙ ccso_frame's body for one plane (EbCcso.c:637-677 with ccso_apply_{luma,chroma}_{mb,sb}_filter, :297-622): the
 * plane at `dst` (device, 8- or 16-bit samples, dst_stride samples) offset in place where the block flag is set,
 * classified on `ext`.  params (host) + flags (host, nvfb * nhfb): those; params = NULL: the state's last search of
 * this plane (stream order, no host wait).  A plane with enable = 0 is left as it is. */
int svtgpu_ccso_apply_plane(SvtGpuCcsoState *s, const uint16_t *ext, int32_t plane, int32_t bit_depth, void *dst,
                            int32_t dst_bits, int32_t dst_stride, const SvtGpuCcsoParams *params,
                            const uint8_t *flags, void *stream);
/* per-block RTCD shims (common_dsp_rtcd.h:1025-1090; host pointers, synchronous) */
uint64_t svtgpu_compute_distortion_block(const uint16_t *org, const int org_stride, const uint16_t *rec16,
                                         const int rec_stride, const int x, const int y,
                                         const int log2_filter_unit_size, const int height, const int width);
void svtgpu_ccso_derive_src_block(const uint16_t *src_y, uint8_t *const src_cls0, uint8_t *const src_cls1,
                                  const int src_y_stride, const int ccso_stride, const int x, const int y,
                                  const int pic_width, const int pic_height, const int y_uv_hscale,
                                  const int y_uv_vscale, const int qstep, const int neg_qstep, const int *src_loc,
                                  const int blk_size, const int edge_clf);
void svtgpu_ccso_filter_block_hbd_with_buf(const uint16_t *src_y, uint16_t *dst_yuv, const uint8_t *src_cls0,
                                           const uint8_t *src_cls1, const int src_y_stride, const int dst_stride,
                                           const int ccso_stride, const int x, const int y, const int pic_width,
                                           const int pic_height, const int8_t *filter_offset, const int blk_size,
                                           const int y_uv_hscale, const int y_uv_vscale, const int max_val,
                                           const uint8_t shift_bits, const uint8_t ccso_bo_only);
void svtgpu_ccso_filter_block_hbd_wo_buf(const uint16_t *src_y, uint16_t *dst_yuv, const int x, const int y,
                                         const int pic_width, const int pic_height, int *src_cls,
                                         const int8_t *offset_buf, const int src_y_stride, const int dst_stride,
                                         const int y_uv_hscale, const int y_uv_vscale, const int thr,
                                         const int neg_thr, const int *src_loc, const int max_val, const int blk_size,
                                         const bool isSingleBand, const uint8_t shift_bits, const int edge_clf,
                                         const uint8_t ccso_bo_only);

#ifdef __cplusplus
}
#endif
#endif /* SVTGPU_H */
