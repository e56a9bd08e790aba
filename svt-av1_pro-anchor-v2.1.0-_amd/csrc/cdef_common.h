// cdef_common.h — CDEF device helpers shared by the search, apply and per-block kernels.
// Semantics follow Source/Lib/Common/Codec/EbCdef.c (reference) line by line where cited.
#pragma once
#include "svtgpu_internal.h"

#define CDEF_VERY_LARGE_V 0x7F7F
#define CDEF_BORDER 2 // the filter reaches +-2 rows/cols (Cdef_Directions, EbCdef.c:99-122)

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// (dy, dx) of svt_aom_eb_cdef_directions[dir][k] (EbCdef.c:99-122), dir in 0..7.  The tables are nibbles of
// 32-bit constants (value + 2 at bits 4*dir): a per-lane direction costs one bit-field extract, where a local
// array indexed by a lane-varying dir would live in scratch memory (one memory load per lookup).
//   dir:        0   1   2   3   4   5   6   7
//   k=0 dy:    -1   0   0   0   1   1   1   1
//   k=1 dy:    -2  -1   0   1   2   2   2   2
//   k=0 dx:     1   1   1   1   1   0   0   0
//   k=1 dx:     2   2   2   2   2   1   0  -1
__device__ __forceinline__ int cdef_dir_dy(int dir, int k) {
    return (int)__builtin_amdgcn_ubfe(k ? 0x44443210u : 0x33332221u, 4 * (dir & 7), 4) - 2;
}
__device__ __forceinline__ int cdef_dir_dx(int dir, int k) {
    return (int)__builtin_amdgcn_ubfe(k ? 0x12344444u : 0x22233333u, 4 * (dir & 7), 4) - 2;
}

__device__ __forceinline__ int msb32_dev(uint32_t v) { return 31 - __clz((int)(v | 1u)); }

// constrain() of EbCdef.c:85-91
__device__ __forceinline__ int cdef_constrain(int diff, int thr, int damping) {
    if (!thr)
        return 0;
    const int shift = max(0, damping - msb32_dev((uint32_t)thr));
    const int ad    = abs(diff);
    const int mag   = min(ad, max(0, thr - (ad >> shift)));
    return diff < 0 ? -mag : mag;
}

// adjust_strength() of EbCdef.c:130-135
__device__ __forceinline__ int cdef_adjust_strength(int strength, int var) {
    const int i = (var >> 6) ? min(msb32_dev((uint32_t)(var >> 6)), 12) : 0;
    return var ? (strength * (4 + i) + 8) >> 4 : 0;
}

// One output sample of svt_cdef_filter_block_c (EbCdef.c:253-300).  `p` points at the sample in
// a 16-bit tile of row stride `ts` with at least CDEF_BORDER samples of context on every side.
__device__ __forceinline__ int cdef_filter_px(const uint16_t *p, int ts, int pri, int sec, int dir, int pdamp,
                                              int sdamp, int coeff_shift) {
    const int  podd = (pri >> coeff_shift) & 1;
    const int  pt0 = podd ? 3 : 4, pt1 = podd ? 3 : 2; // svt_aom_eb_cdef_pri_taps
    const int  x   = (int16_t)p[0];
    int16_t    sum = 0;
    int        hi = x, lo = x;
    const int  ds0 = (dir + 2) & 7, ds1 = (dir + 6) & 7;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int op  = cdef_dir_dy(dir, k) * ts + cdef_dir_dx(dir, k);
        const int o0  = cdef_dir_dy(ds0, k) * ts + cdef_dir_dx(ds0, k);
        const int o1  = cdef_dir_dy(ds1, k) * ts + cdef_dir_dx(ds1, k);
        const int pw  = k ? pt1 : pt0;
        const int sw  = k ? 1 : 2; // svt_aom_eb_cdef_sec_taps
        const int v[6] = {(int16_t)p[op], (int16_t)p[-op], (int16_t)p[o0], (int16_t)p[-o0], (int16_t)p[o1], (int16_t)p[-o1]};
        sum += (int16_t)(pw * cdef_constrain(v[0] - x, pri, pdamp));
        sum += (int16_t)(pw * cdef_constrain(v[1] - x, pri, pdamp));
#pragma unroll
        for (int t = 0; t < 6; t++) {
            if (v[t] != CDEF_VERY_LARGE_V)
                hi = max(hi, v[t]);
            lo = min(lo, v[t]);
        }
#pragma unroll
        for (int t = 2; t < 6; t++) sum += (int16_t)(sw * cdef_constrain(v[t] - x, sec, sdamp));
    }
    int y = x + ((8 + sum - (sum < 0)) >> 4);
    return y < lo ? lo : (y > hi ? hi : y);
}

// Sum of a value over each aligned 16-lane row of the wave (result in every lane of the row),
// DPP only: quad xor1, quad xor2, row_half_mirror, row_mirror.
__device__ __forceinline__ uint32_t row16_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return v;
}

// SSIM-like luma term of dist_8xn_16bit_c / dist_8xn_8bit_c (EbEncCdef.c:23-48, :76-101).
// Operand order and IEEE double ops are those of the reference; the library is built with
// -ffp-contract=off so no FMA contraction can change the rounding.
__device__ __forceinline__ uint64_t cdef_luma_dist(uint64_t sum_s, uint64_t sum_d, uint64_t sum_s2, uint64_t sum_d2,
                                                   uint64_t sse, int coeff_shift) {
    const uint64_t svar = sum_s2 - ((sum_s * sum_s + 32) >> 6);
    const uint64_t dvar = sum_d2 - ((sum_d * sum_d + 32) >> 6);
    const double   num  = (double)sse * .5 * (double)(svar + dvar + (uint64_t)(400 << 2 * coeff_shift));
    const double   den  = sqrt((double)(20000 << 4 * coeff_shift) + (double)svar * (double)dvar);
    return (uint64_t)floor(.5 + num / den);
}
