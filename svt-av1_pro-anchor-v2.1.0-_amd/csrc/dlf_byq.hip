// dlf_byq.hip — loop-filter levels from the quantizer (LPF_PICK_FROM_Q), host logic of the C ABI.
//
// ≙ svt_av1_pick_filter_level_by_q (Source/Lib/Encoder/Codec/EbDeblockingFilter.c:1036-1125) and qp_based_dlf_param
// (:992-1031).  A handful of integer operations per frame: nothing here is worth a launch, and the result feeds
// svtgpu_dlf_frame / svtgpu_dlf_frame_to as the LfParams levels.
#include "av1_ac_quant.h"
#include "svtgpu_internal.h"

namespace {
// EbDeblockingFilter.c:25-29, indexed by ResolutionRange (240p .. 8K) and DlfCtrls.zero_filter_strength_lvl
constexpr int32_t  kInterFrameMult[7] = {6017, 6017, 6017, 12034, 12034, 12034, 12034};
constexpr uint32_t kZeroStrengthTh[4][7] = {{0, 0, 0, 0, 0, 0, 0},
                                            {100, 200, 500, 800, 1000, 1300, 1600},
                                            {900, 1000, 2000, 3000, 4000, 6000, 7000},
                                            {6000, 7000, 8000, 9000, 10000, 20000, 30000}};
constexpr int kMaxLevel = 63; // MAX_LOOP_FILTER

int32_t round_shift(int64_t v, int n) { return (int32_t)((v + ((1 << n) >> 1)) >> n); } // ROUND_POWER_OF_TWO
int32_t clamp_level(int32_t v) { return v < 0 ? 0 : v > kMaxLevel ? kMaxLevel : v; }
int     bd_index(int32_t bd) { return bd == 8 ? 0 : bd == 10 ? 1 : bd == 12 ? 2 : -1; }

// the level guess both paths share; `inter_mult` is the 8-bit inter-frame slope (qp_based: 6017 always)
int32_t level_guess(int32_t bd, int32_t q, int32_t frame_type, int32_t inter_mult) {
    int32_t g;
    if (bd == 8)
        g = frame_type == 0 ? round_shift((int64_t)q * 17563 - 421574, 18) : round_shift((int64_t)q * inter_mult + 650707, 18);
    else if (bd == 10)
        g = round_shift((int64_t)q * 20723 + 4060632, 20);
    else
        g = round_shift((int64_t)q * 20723 + 16242526, 22);
    if (bd != 8 && frame_type == 0) g -= 4; // high bit depth key frames
    return g;
}
} // namespace

extern "C" int svtgpu_dlf_pick_by_q(const SvtGpuDlfByQ *in, int32_t filter_level[4]) {
    if (!in || !filter_level || bd_index(in->bit_depth) < 0 || in->base_q_idx < 0 || in->base_q_idx > 255 ||
        in->input_resolution < 0 || in->input_resolution > 6 || in->zero_filter_strength_lvl < 0 ||
        in->zero_filter_strength_lvl > 3 || in->nref < 0 || in->nref > 7 || in->b64_count < 0 ||
        (in->b64_count && !in->me_sad))
        return SVTGPU_ERR_INVALID_ARG;
    int32_t min_ref[4] = {kMaxLevel, kMaxLevel, kMaxLevel, kMaxLevel}; // :1043-1063
    for (int r = 0; r < in->nref; r++)
        for (int k = 0; k < 4; k++) min_ref[k] = in->ref_levels[r][k] < min_ref[k] ? in->ref_levels[r][k] : min_ref[k];
    const int32_t q     = kAv1AcQuant[bd_index(in->bit_depth)][in->base_q_idx];
    int32_t       guess = level_guess(in->bit_depth, q, in->frame_type, kInterFrameMult[in->input_resolution]);
    int32_t       guess_uv = guess / 2;
    if (in->slice_type != 2) { // not I_SLICE: shut the filter on static content (:1092-1107)
        const uint32_t th = kZeroStrengthTh[in->zero_filter_strength_lvl][in->input_resolution] *
                            (uint32_t)(in->temporal_layer_index + 1);
        if (th) {
            uint32_t total = 0; // uint32 running sum, as the reference keeps it
            for (int b = 0; b < in->b64_count; b++) total += in->me_sad[b];
            const uint32_t avg = in->b64_count ? total / (uint32_t)in->b64_count : 0;
            if (avg < th) guess = 0;
            if (avg < th * 2) guess_uv = 0;
        }
    }
    const bool base_layer = in->ppcs_temporal_layer_index == 0; // :1109-1124
    filter_level[0] = min_ref[0] || base_layer ? clamp_level(guess) : 0;
    filter_level[1] = min_ref[1] || base_layer ? clamp_level(guess) : 0;
    filter_level[2] = min_ref[2] || base_layer ? clamp_level(guess_uv) : 0;
    filter_level[3] = min_ref[3] || base_layer ? clamp_level(guess_uv) : 0;
    return SVTGPU_OK;
}

extern "C" int svtgpu_dlf_qp_based_param(int32_t bit_depth, int32_t base_q_idx, int32_t frame_type,
                                         int32_t *filter_level_y, int32_t *filter_level_uv) {
    if (!filter_level_y || !filter_level_uv || bd_index(bit_depth) < 0 || base_q_idx < 0 || base_q_idx > 255)
        return SVTGPU_ERR_INVALID_ARG;
    int32_t g = level_guess(bit_depth, kAv1AcQuant[bd_index(bit_depth)][base_q_idx], frame_type, 6017);
    g         = g > 2 ? g - 2 : g > 1 ? g - 1 : g; // :1024
    *filter_level_y  = clamp_level(g);
    *filter_level_uv = clamp_level(g > 1 ? g / 2 : g);
    return SVTGPU_OK;
}
