// frame_ops.hip — the frame-buffer work around the in-loop filter path on gfx950.
//
//   bit-depth conversion   svt_convert_8bit_to_16bit_c / svt_convert_16bit_to_8bit_c
//                          (Source/Lib/Common/C_DEFAULT/EbPackUnPack_C.c:270-283; RTCD common_dsp_rtcd.h:154-156), used
//                          per picture by svt_convert_pic_8bit_to_16bit (EbRestProcess.c:235-272, the 16-bit pipeline's
//                          8-bit input) and the non-reference 16 -> 8 copy-back (EbRestProcess.c:670-697)
//   reference padding      svt_aom_generate_padding / svt_aom_generate_padding16_bit (Common/Codec/EbMcp.c:95-150,
//                          201-240; pad_ref_and_set_flags, EbEncDecProcess.c:1589-1660): replicate the first / last
//                          sample of every picture row over the side borders, then copy the first / last padded row
//                          (the whole stride) over the top / bottom borders
//   frame extension        svt_extend_frame (Common/Codec/EbRestoration.c:160-203): the same replication over a border
//                          around the visible area, columns [-border_horz, width + border_horz) only
// All three are one pass over the bytes they must touch: 16-byte vector loads/stores per lane on the aligned interior
// (the device frames' rows are 256-B aligned), scalar edges; the padding kernels write only the borders.
#include <cstring>

#include "svtgpu_internal.h"

namespace {

// ---- conversion: 16 samples per lane ----
template <typename S, typename D>
__global__ __launch_bounds__(256) void convert_kernel(const S *src, int ss, D *dst, int ds, int w, int h) {
    const int y = blockIdx.y, x0 = 16 * (blockIdx.x * 256 + threadIdx.x);
    if (y >= h || x0 >= w) return;
    const S *s = src + (size_t)y * ss + x0;
    D       *d = dst + (size_t)y * ds + x0;
    const bool vec = x0 + 16 <= w && !(((uintptr_t)s) & 15) && !(((uintptr_t)d) & 15);
    if (vec && sizeof(S) == 1) { // 8 -> 16: one 16-B load, two 16-B stores
        const uint4 v = *(const uint4 *)s;
        const uint32_t in[4] = {v.x, v.y, v.z, v.w};
        uint32_t       o[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            o[2 * k]     = __builtin_amdgcn_perm(0u, in[k], 0x0c010c00u); // bytes 0,1 -> u16 lanes
            o[2 * k + 1] = __builtin_amdgcn_perm(0u, in[k], 0x0c030c02u);
        }
        ((uint4 *)d)[0] = make_uint4(o[0], o[1], o[2], o[3]);
        ((uint4 *)d)[1] = make_uint4(o[4], o[5], o[6], o[7]);
    } else if (vec) { // 16 -> 8: two 16-B loads, one 16-B store (the low byte of every sample)
        const uint4 a = ((const uint4 *)s)[0], b = ((const uint4 *)s)[1];
        const uint32_t in[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t       o[4];
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = __builtin_amdgcn_perm(in[2 * k + 1], in[2 * k], 0x06040200u);
        *(uint4 *)d = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        for (int k = 0; k < 16 && x0 + k < w; k++) d[k] = (D)s[k];
    }
}

// ---- padding (generate_padding semantics): rows [0, ph + h + ph) of a buffer whose visible area starts at (pw, ph) ----
template <typename T>
__global__ __launch_bounds__(256) void pad_kernel(T *buf, int stride, int w, int h, int pw, int ph) {
    const int r = blockIdx.x; // buffer row
    T        *row = buf + (size_t)r * stride;
    if (r >= ph && r < ph + h) { // a visible row: its side borders
        const T a = row[pw], b = row[pw + w - 1];
        for (int i = threadIdx.x; i < pw; i += blockDim.x) row[i] = a, row[pw + w + i] = b;
        return;
    }
    // a top / bottom border row: the whole stride of the first / last visible row after its side padding
    const int sr = r < ph ? ph : ph + h - 1;
    const T  *s  = buf + (size_t)sr * stride;
    for (int i = threadIdx.x; i < stride; i += blockDim.x)
        row[i] = i < pw ? s[pw] : (i >= pw + w && i < pw + w + pw) ? s[pw + w - 1] : s[i];
}

// ---- extension (svt_extend_frame semantics): data = first visible sample ----
template <typename T>
__global__ __launch_bounds__(256) void extend_kernel(T *data, int stride, int w, int h, int bh, int bv) {
    const int r = (int)blockIdx.x - bv; // visible row index in [-bv, h + bv)
    T        *row = data + (ptrdiff_t)r * stride;
    const T  *s   = data + (ptrdiff_t)min(max(r, 0), h - 1) * stride;
    if (r >= 0 && r < h) {
        const T a = s[0], b = s[w - 1];
        for (int i = threadIdx.x; i < bh; i += blockDim.x) row[-bh + i] = a, row[w + i] = b;
        return;
    }
    for (int i = threadIdx.x - bh; i < w + bh; i += blockDim.x) row[i] = s[min(max(i, 0), w - 1)];
}

int convert_dev(const void *src, int sbits, int ss, void *dst, int dbits, int ds, int w, int h, hipStream_t st) {
    if (w <= 0 || h <= 0) return SVTGPU_OK;
    const dim3 grid((w + 16 * 256 - 1) / (16 * 256), h);
    if (sbits == 8 && dbits == 16)
        hipLaunchKernelGGL((convert_kernel<uint8_t, uint16_t>), grid, dim3(256), 0, st, (const uint8_t *)src, ss,
                           (uint16_t *)dst, ds, w, h);
    else if (sbits == 16 && dbits == 8)
        hipLaunchKernelGGL((convert_kernel<uint16_t, uint8_t>), grid, dim3(256), 0, st, (const uint16_t *)src, ss,
                           (uint8_t *)dst, ds, w, h);
    else
        return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

int pad_dev(void *buf, int bits, int stride, int w, int h, int pw, int ph, hipStream_t st) {
    if (w <= 0 || h <= 0 || pw < 0 || ph < 0 || stride < w + 2 * pw) return SVTGPU_ERR_INVALID_ARG;
    if (bits == 8)
        hipLaunchKernelGGL(pad_kernel<uint8_t>, dim3(h + 2 * ph), dim3(256), 0, st, (uint8_t *)buf, stride, w, h, pw, ph);
    else if (bits == 16)
        hipLaunchKernelGGL(pad_kernel<uint16_t>, dim3(h + 2 * ph), dim3(256), 0, st, (uint16_t *)buf, stride, w, h, pw,
                           ph);
    else
        return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

int extend_dev(void *data, int bits, int stride, int w, int h, int bh, int bv, hipStream_t st) {
    if (w <= 0 || h <= 0 || bh < 0 || bv < 0) return SVTGPU_ERR_INVALID_ARG;
    if (bits == 8)
        hipLaunchKernelGGL(extend_kernel<uint8_t>, dim3(h + 2 * bv), dim3(256), 0, st, (uint8_t *)data, stride, w, h, bh,
                           bv);
    else if (bits == 16)
        hipLaunchKernelGGL(extend_kernel<uint16_t>, dim3(h + 2 * bv), dim3(256), 0, st, (uint16_t *)data, stride, w, h,
                           bh, bv);
    else
        return SVTGPU_ERR_INVALID_ARG;
    HIP_TRY(hipGetLastError());
    return SVTGPU_OK;
}

// host staging of a strided region [first byte, last byte] for the synchronous shims
struct HostSpan {
    uint8_t *d = nullptr;
    ~HostSpan() { (void)hipFree(d); }
};

} // namespace

// ---- device-pointer entry points ----
extern "C" int svtgpu_convert_plane(const void *src, int32_t src_bits, int32_t src_stride, void *dst, int32_t dst_bits,
                                    int32_t dst_stride, int32_t width, int32_t height, void *stream) {
    if (!src || !dst) return SVTGPU_ERR_INVALID_ARG;
    return convert_dev(src, src_bits, src_stride, dst, dst_bits, dst_stride, width, height,
                       stream ? (hipStream_t)stream : svtgpu_default_stream());
}

extern "C" int svtgpu_pad_plane(void *buf, int32_t bits, int32_t stride, int32_t width, int32_t height,
                                int32_t pad_width, int32_t pad_height, void *stream) {
    if (!buf) return SVTGPU_ERR_INVALID_ARG;
    return pad_dev(buf, bits, stride, width, height, pad_width, pad_height,
                   stream ? (hipStream_t)stream : svtgpu_default_stream());
}

extern "C" int svtgpu_extend_plane(void *data, int32_t bits, int32_t stride, int32_t width, int32_t height,
                                   int32_t border_horz, int32_t border_vert, void *stream) {
    if (!data) return SVTGPU_ERR_INVALID_ARG;
    return extend_dev(data, bits, stride, width, height, border_horz, border_vert,
                      stream ? (hipStream_t)stream : svtgpu_default_stream());
}

// svt_convert_pic_8bit_to_16bit (EbRestProcess.c:235-272) / the 16 -> 8 copy-back (:670-697) of device frames
extern "C" int svtgpu_frame_convert(const SvtGpuFrame *src, SvtGpuFrame *dst, void *stream) {
    if (!src || !dst || src->width != dst->width || src->height != dst->height) return SVTGPU_ERR_INVALID_ARG;
    const int sb = src->bytes_per_sample * 8, db = dst->bytes_per_sample * 8;
    if (sb == db) return SVTGPU_ERR_INVALID_ARG;
    hipStream_t st = pick_stream(dst->ctx, stream);
    for (int p = 0; p < 3; p++)
        if (int rc = convert_dev(src->plane[p], sb, src->stride[p], dst->plane[p], db, dst->stride[p], src->pw[p],
                                 src->ph[p], st))
            return rc;
    return SVTGPU_OK;
}

// ---- RTCD-compatible shims (synchronous, host pointers) ----
namespace {
template <typename T>
T *stage_in(hipStream_t st, HostSpan &sp, const T *h, size_t first, size_t n_elems) { // [h + first, + n_elems)
    HIP_OR_DIE(hipMalloc(&sp.d, n_elems * sizeof(T)));
    HIP_OR_DIE(hipMemcpyAsync(sp.d, h + first, n_elems * sizeof(T), hipMemcpyHostToDevice, st));
    return (T *)sp.d;
}
template <typename T>
void stage_out(hipStream_t st, T *h, size_t first, const HostSpan &sp, size_t n_elems) {
    HIP_OR_DIE(hipMemcpyAsync(h + first, sp.d, n_elems * sizeof(T), hipMemcpyDeviceToHost, st));
    HIP_OR_DIE(hipStreamSynchronize(st));
}
} // namespace

// svt_convert_8bit_to_16bit (common_dsp_rtcd.h:154)
extern "C" void svtgpu_convert_8bit_to_16bit(uint8_t *src, uint32_t src_stride, uint16_t *dst, uint32_t dst_stride,
                                             uint32_t width, uint32_t height) {
    if (!width || !height) return;
    hipStream_t st = svtgpu_shim_stream();
    HostSpan    a, b;
    const size_t ns = (size_t)(height - 1) * src_stride + width, nd = (size_t)(height - 1) * dst_stride + width;
    uint8_t     *ds = stage_in(st, a, src, 0, ns);
    uint16_t    *dd = stage_in(st, b, dst, 0, nd); // the samples between rows stay as they were
    HIP_OR_DIE(convert_dev(ds, 8, (int)src_stride, dd, 16, (int)dst_stride, (int)width, (int)height, st) ? hipErrorUnknown
                                                                                                         : hipSuccess);
    stage_out(st, dst, 0, b, nd);
}

// svt_convert_16bit_to_8bit (common_dsp_rtcd.h:156)
extern "C" void svtgpu_convert_16bit_to_8bit(uint16_t *src, uint32_t src_stride, uint8_t *dst, uint32_t dst_stride,
                                             uint32_t width, uint32_t height) {
    if (!width || !height) return;
    hipStream_t st = svtgpu_shim_stream();
    HostSpan    a, b;
    const size_t ns = (size_t)(height - 1) * src_stride + width, nd = (size_t)(height - 1) * dst_stride + width;
    uint16_t    *ds = stage_in(st, a, src, 0, ns);
    uint8_t     *dd = stage_in(st, b, dst, 0, nd);
    HIP_OR_DIE(convert_dev(ds, 16, (int)src_stride, dd, 8, (int)dst_stride, (int)width, (int)height, st) ? hipErrorUnknown
                                                                                                         : hipSuccess);
    stage_out(st, dst, 0, b, nd);
}

// svt_aom_generate_padding (EbMcp.h:46): the buffer holds (h + 2 ph) rows of `stride` samples
extern "C" void svtgpu_aom_generate_padding(uint8_t *src_pic, uint32_t src_stride, uint32_t original_src_width,
                                            uint32_t original_src_height, uint32_t padding_width,
                                            uint32_t padding_height) {
    if (!src_pic) return;
    hipStream_t  st = svtgpu_shim_stream();
    HostSpan     a;
    const size_t n  = (size_t)(original_src_height + 2 * padding_height) * src_stride;
    uint8_t     *d  = stage_in(st, a, src_pic, 0, n);
    HIP_OR_DIE(pad_dev(d, 8, (int)src_stride, (int)original_src_width, (int)original_src_height, (int)padding_width,
                       (int)padding_height, st)
                   ? hipErrorUnknown
                   : hipSuccess);
    stage_out(st, src_pic, 0, a, n);
}

// svt_aom_generate_padding16_bit (EbMcp.h:49)
extern "C" void svtgpu_aom_generate_padding16_bit(uint16_t *src_pic, uint32_t src_stride, uint32_t original_src_width,
                                                  uint32_t original_src_height, uint32_t padding_width,
                                                  uint32_t padding_height) {
    hipStream_t  st = svtgpu_shim_stream();
    HostSpan     a;
    const size_t n  = (size_t)(original_src_height + 2 * padding_height) * src_stride;
    uint16_t    *d  = stage_in(st, a, src_pic, 0, n);
    HIP_OR_DIE(pad_dev(d, 16, (int)src_stride, (int)original_src_width, (int)original_src_height, (int)padding_width,
                       (int)padding_height, st)
                   ? hipErrorUnknown
                   : hipSuccess);
    stage_out(st, src_pic, 0, a, n);
}

// svt_extend_frame (EbRestoration.c:197; highbd data is a CONVERT_TO_BYTEPTR pointer)
extern "C" void svtgpu_extend_frame(uint8_t *data, int32_t width, int32_t height, int32_t stride, int32_t border_horz,
                                    int32_t border_vert, int32_t highbd) {
    hipStream_t st    = svtgpu_shim_stream();
    const size_t rows = (size_t)height + 2 * border_vert;
    // the touched span: from (-bv, -bh) to (h + bv - 1, w + bh - 1)
    const ptrdiff_t first = -(ptrdiff_t)border_vert * stride - border_horz;
    const size_t    n     = (rows - 1) * (size_t)stride + (size_t)(width + 2 * border_horz);
    HostSpan        a;
    if (highbd) {
        uint16_t *h = (uint16_t *)((uintptr_t)data << 1) + first; // CONVERT_TO_SHORTPTR
        uint16_t *d = stage_in(st, a, h, 0, n);
        HIP_OR_DIE(extend_dev(d - first, 16, stride, width, height, border_horz, border_vert, st) ? hipErrorUnknown
                                                                                                   : hipSuccess);
        stage_out(st, h, 0, a, n);
    } else {
        uint8_t *h = data + first;
        uint8_t *d = stage_in(st, a, h, 0, n);
        HIP_OR_DIE(extend_dev(d - first, 8, stride, width, height, border_horz, border_vert, st) ? hipErrorUnknown
                                                                                                  : hipSuccess);
        stage_out(st, h, 0, a, n);
    }
}
