"""ctypes binding of libsvtgpu (the MI355X C ABI declared in include/svtgpu.h).

Host-side mirror of the reference's CDEF frame pipeline surface (EbCdefProcess.c /
EbEncCdef.c): search -> pick -> apply on device-resident 4:2:0 frames.  This module is what
tests/ and bench.py call; it never falls back to a CPU path — if the HIP library is missing or no
gfx950 device is visible, it raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVTGPU_LIB") or os.path.join(_HERE, "lib", "libsvtgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "svtgpu.h")

SVTGPU_OK = 0
TOTAL_STRENGTHS = 64
MAX_STRENGTHS = 16


class CdefList(ctypes.Structure):
    _fields_ = [("by", ctypes.c_uint8), ("bx", ctypes.c_uint8)]


class CdefControls(ctypes.Structure):
    """SvtGpuCdefControls (mirror of CdefControls, EbPictureControlSet.h:592-628)."""
    _fields_ = [
        ("first_pass_fs_num", ctypes.c_uint8),
        ("default_second_pass_fs_num", ctypes.c_uint8),
        ("default_first_pass_fs", ctypes.c_uint8 * TOTAL_STRENGTHS),
        ("default_second_pass_fs", ctypes.c_uint8 * TOTAL_STRENGTHS),
        ("default_first_pass_fs_uv", ctypes.c_int8 * TOTAL_STRENGTHS),
        ("default_second_pass_fs_uv", ctypes.c_int8 * TOTAL_STRENGTHS),
        ("subsampling_factor", ctypes.c_uint8),
        ("zero_fs_cost_bias", ctypes.c_uint16),
        ("use_reference_cdef_fs", ctypes.c_int8),
        ("pred_y_f", ctypes.c_int8),
        ("pred_uv_f", ctypes.c_int8),
    ]

    def strengths(self):
        n1, n2 = self.first_pass_fs_num, self.default_second_pass_fs_num
        return list(self.default_first_pass_fs[:n1]) + list(self.default_second_pass_fs[:n2])


class CdefParams(ctypes.Structure):
    """SvtGpuCdefParams (mirror of CdefParams, EbAv1Structs.h:359-369)."""
    _fields_ = [
        ("cdef_damping", ctypes.c_uint8),
        ("cdef_bits", ctypes.c_uint8),
        ("cdef_y_strength", ctypes.c_uint8 * MAX_STRENGTHS),
        ("cdef_uv_strength", ctypes.c_uint8 * MAX_STRENGTHS),
    ]

    def as_tuple(self):
        nb = 1 << self.cdef_bits
        return (self.cdef_damping, self.cdef_bits, tuple(self.cdef_y_strength[:nb]),
                tuple(self.cdef_uv_strength[:nb]))


class LfMi(ctypes.Structure):
    """SvtGpuLfMi: the MbModeInfo.block_mi fields the deblocking filter reads (one per 4x4 mi)."""
    _fields_ = [("bsize", ctypes.c_uint8), ("tx_depth", ctypes.c_uint8), ("skip", ctypes.c_uint8),
                ("ref_frame0", ctypes.c_int8), ("mode", ctypes.c_uint8), ("segment_id", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 2)]


LF_MI_DTYPE = np.dtype([("bsize", np.uint8), ("tx_depth", np.uint8), ("skip", np.uint8), ("ref_frame0", np.int8),
                        ("mode", np.uint8), ("segment_id", np.uint8), ("pad", np.uint8, 2)])


class LfParams(ctypes.Structure):
    """SvtGpuLfParams (struct LoopFilter, EbDefinitions.h:1903-1920, + segmentation features)."""
    _fields_ = [
        ("filter_level", ctypes.c_int32 * 2),
        ("filter_level_u", ctypes.c_int32),
        ("filter_level_v", ctypes.c_int32),
        ("sharpness_level", ctypes.c_int32),
        ("mode_ref_delta_enabled", ctypes.c_uint8),
        ("ref_deltas", ctypes.c_int8 * 8),
        ("mode_deltas", ctypes.c_int8 * 2),
        ("segmentation_enabled", ctypes.c_uint8),
        ("seg_feature_data", (ctypes.c_int16 * 8) * 8),
        ("seg_feature_enabled", (ctypes.c_int16 * 8) * 8),
    ]

    def levels(self):
        return (self.filter_level[0], self.filter_level[1], self.filter_level_u, self.filter_level_v)

    @classmethod
    def make(cls, fl0, fl1, flu, flv, sharpness=0, ref_deltas=None, mode_deltas=None, seg_enabled=None,
             seg_data=None):
        """Build from plain values; ref_deltas/mode_deltas given => mode_ref_delta_enabled."""
        p = cls()
        p.filter_level[0], p.filter_level[1], p.filter_level_u, p.filter_level_v = fl0, fl1, flu, flv
        p.sharpness_level = sharpness
        if ref_deltas is not None:
            p.mode_ref_delta_enabled = 1
            for i, v in enumerate(ref_deltas):
                p.ref_deltas[i] = int(v)
            for i, v in enumerate(mode_deltas if mode_deltas is not None else (0, 0)):
                p.mode_deltas[i] = int(v)
        if seg_enabled is not None:
            p.segmentation_enabled = 1
            for s in range(8):
                for f in range(8):
                    p.seg_feature_enabled[s][f] = int(seg_enabled[s][f])
                    p.seg_feature_data[s][f] = int(seg_data[s][f])
        return p


class DlfByQ(ctypes.Structure):
    """SvtGpuDlfByQ: what svt_av1_pick_filter_level_by_q reads (EbDeblockingFilter.c:1036-1125)."""
    _fields_ = [("bit_depth", ctypes.c_int32), ("base_q_idx", ctypes.c_int32), ("frame_type", ctypes.c_int32),
                ("slice_type", ctypes.c_int32), ("temporal_layer_index", ctypes.c_int32),
                ("ppcs_temporal_layer_index", ctypes.c_int32), ("input_resolution", ctypes.c_int32),
                ("zero_filter_strength_lvl", ctypes.c_int32), ("b64_count", ctypes.c_int32),
                ("me_sad", ctypes.POINTER(ctypes.c_uint32)), ("nref", ctypes.c_int32),
                ("ref_levels", (ctypes.c_int32 * 4) * 7)]


def dlf_pick_by_q(bit_depth, base_q_idx, frame_type, slice_type, temporal_layer_index, ppcs_temporal_layer_index,
                  input_resolution, zero_filter_strength_lvl, me_sad, ref_levels):
    """svtgpu_dlf_pick_by_q (host): LfParams levels (y0, y1, u, v) from the quantizer, no search."""
    me = np.ascontiguousarray(me_sad, np.uint32)
    a = DlfByQ(bit_depth, base_q_idx, frame_type, slice_type, temporal_layer_index, ppcs_temporal_layer_index,
               input_resolution, zero_filter_strength_lvl, len(me), me.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
               len(ref_levels))
    for i, lv in enumerate(ref_levels):
        for k in range(4):
            a.ref_levels[i][k] = int(lv[k])
    out = (ctypes.c_int32 * 4)()
    check(lib().svtgpu_dlf_pick_by_q(ctypes.byref(a), out))
    return tuple(out)


def dlf_qp_based_param(bit_depth, base_q_idx, frame_type):
    y, uv = ctypes.c_int32(), ctypes.c_int32()
    check(lib().svtgpu_dlf_qp_based_param(bit_depth, base_q_idx, frame_type, ctypes.byref(y), ctypes.byref(uv)))
    return y.value, uv.value


class RestUnit(ctypes.Structure):
    """SvtGpuRestUnit (RestorationUnitInfo, EbRestoration.h:169-188)."""
    _fields_ = [("type", ctypes.c_int32), ("vfilter", ctypes.c_int16 * 8), ("hfilter", ctypes.c_int16 * 8),
                ("ep", ctypes.c_int32), ("xqd", ctypes.c_int32 * 2)]


REST_UNIT_DTYPE = np.dtype([("type", np.int32), ("vfilter", np.int16, 8), ("hfilter", np.int16, 8), ("ep", np.int32),
                            ("xqd", np.int32, 2)])


def rest_units_from_rows(rows):
    """[n][20] int32 rows {type, vfilter[8], hfilter[8], ep, xqd0, xqd1} -> REST_UNIT_DTYPE array."""
    rows = np.asarray(rows)
    u = np.zeros(len(rows), REST_UNIT_DTYPE)
    u["type"] = rows[:, 0]
    u["vfilter"] = rows[:, 1:9]
    u["hfilter"] = rows[:, 9:17]
    u["ep"] = rows[:, 17]
    u["xqd"] = rows[:, 18:20]
    return u


class LrSearchControls(ctypes.Structure):
    """SvtGpuLrSearchControls (WnFilterCtrls / SgFilterCtrls + Macroblock rate fields)."""
    _fields_ = [("wn_enabled", ctypes.c_int32), ("wn_use_chroma", ctypes.c_int32), ("wn_filter_tap_lvl", ctypes.c_int32),
                ("wn_use_refinement", ctypes.c_int32), ("wn_max_one_refinement_step", ctypes.c_int32),
                ("sg_enabled", ctypes.c_int32), ("sg_use_chroma", ctypes.c_int32),
                ("sg_start_ep", ctypes.c_int32 * 2), ("sg_end_ep", ctypes.c_int32 * 2),
                ("sg_ep_inc", ctypes.c_int32 * 2), ("sg_refine", ctypes.c_int32 * 2), ("rdmult", ctypes.c_int32),
                ("switchable_restore_cost", ctypes.c_int32 * 3), ("wiener_restore_cost", ctypes.c_int32 * 2),
                ("sgrproj_restore_cost", ctypes.c_int32 * 2)]


LR_PROFILE_DTYPE = np.dtype([("launches", np.int32, 6), ("ms", np.float32, 6), ("bytes", np.float64, 6),
                             ("searches", np.int32), ("ms_events", np.float32, 6)], align=True)
LR_UNIT_SEARCH_DTYPE = np.dtype([("sse", np.int64, 3), ("wiener", REST_UNIT_DTYPE), ("sgrproj", REST_UNIT_DTYPE)],
                                align=True)


class CcsoParams(ctypes.Structure):
    """SvtGpuCcsoParams: one plane of FrameHeader.ccso_info (EbAv1Structs.h:407-427)."""
    _fields_ = [("enable", ctypes.c_uint8), ("bo_only", ctypes.c_uint8), ("quant_idx", ctypes.c_uint8),
                ("ext_filter_support", ctypes.c_uint8), ("max_band_log2", ctypes.c_uint8), ("edge_clf", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8 * 2), ("filter_offset", ctypes.c_int8 * 2048)]

    FIELDS = ("enable", "bo_only", "quant_idx", "ext_filter_support", "max_band_log2", "edge_clf")

    @classmethod
    def make(cls, fields, lut):
        p = cls()
        for n, v in zip(cls.FIELDS, fields):
            setattr(p, n, int(v))
        ctypes.memmove(p.filter_offset, np.ascontiguousarray(lut, dtype=np.int8).ctypes.data, 2048)
        return p

    def fields(self):
        return tuple(int(getattr(self, n)) for n in self.FIELDS)

    def lut(self):
        return np.frombuffer(bytes(self.filter_offset), dtype=np.int8).copy()


class ConvolveParams(ctypes.Structure):
    """SvtGpuConvolveParams: the reference's ConvolveParams layout (EbDefinitions.h:577-590)."""
    _fields_ = [("ref", ctypes.c_int32), ("do_average", ctypes.c_int32), ("dst", ctypes.c_void_p),
                ("dst_stride", ctypes.c_int32), ("round_0", ctypes.c_int32), ("round_1", ctypes.c_int32),
                ("plane", ctypes.c_int32), ("is_compound", ctypes.c_int32), ("use_jnt_comp_avg", ctypes.c_int32),
                ("fwd_offset", ctypes.c_int32), ("bck_offset", ctypes.c_int32),
                ("use_dist_wtd_comp_avg", ctypes.c_int32)]


class SgrParams(ctypes.Structure):
    """SvtGpuSgrParams: the reference's SgrParamsType (EbDefinitions.h:1768-1771)."""
    _fields_ = [("r", ctypes.c_int32 * 2), ("s", ctypes.c_int32 * 2)]


MD_SIZES = [(4, 4), (4, 8), (8, 4), (8, 8), (8, 16), (16, 8), (16, 16), (16, 32), (32, 16), (32, 32), (32, 64),
            (64, 32), (64, 64), (64, 128), (128, 64), (128, 128), (4, 16), (16, 4), (8, 32), (32, 8), (16, 64),
            (64, 16)]
MD_BLOCKS = 849

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_U64 = ctypes.c_uint64
_U8P = ctypes.POINTER(ctypes.c_uint8)
_LPF8 = (None, [_P, _I32, _P, _P, _P])
_LPF16 = (None, [_P, _I32, _P, _P, _P, _I32])
_SIGS = {
    "svtgpu_device_available": (ctypes.c_int, []),
    "svtgpu_version": (ctypes.c_char_p, []),
    "svtgpu_abi_version": (_I32, []),
    "svtgpu_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "svtgpu_context_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "svtgpu_context_destroy": (None, [_P]),
    "svtgpu_context_stream": (_P, [_P]),
    "svtgpu_synchronize": (ctypes.c_int, [_P, _P]),
    "svtgpu_stream_create": (ctypes.c_int, [_P, _I32, ctypes.POINTER(_P)]),
    "svtgpu_stream_destroy": (None, [_P]),
    "svtgpu_frame_create": (ctypes.c_int, [_P, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_frame_destroy": (None, [_P]),
    "svtgpu_frame_stride": (_I32, [_P, ctypes.c_int]),
    "svtgpu_frame_plane_ptr": (_P, [_P, ctypes.c_int]),
    "svtgpu_frame_upload": (ctypes.c_int, [_P, ctypes.c_int, _P, _I32, _P]),
    "svtgpu_frame_download": (ctypes.c_int, [_P, ctypes.c_int, _P, _I32, _P]),
    "svtgpu_frame_upload_rect": (ctypes.c_int, [_P, ctypes.c_int, _P, _I32, _P, _P]),
    "svtgpu_frame_copy": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_find_dir": (ctypes.c_uint8, [_P, _I32, ctypes.POINTER(_I32), _I32]),
    "svtgpu_cdef_find_dir_dual": (None, [_P, _P, ctypes.c_int, ctypes.POINTER(_I32), ctypes.POINTER(_I32), _I32,
                                         ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint8)]),
    "svtgpu_cdef_filter_block": (None, [_P, _P, _I32, _P, _I32, _I32, _I32, _I32, _I32, _I32, _I32, ctypes.c_uint8]),
    "svtgpu_compute_cdef_dist_16bit": (_U64, [_P, _I32, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_uint8]),
    "svtgpu_compute_cdef_dist_8bit": (_U64, [_P, _I32, _P, _P, _I32, _I32, _I32, _I32, ctypes.c_uint8]),
    "svtgpu_search_one_dual": (_U64, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                      ctypes.POINTER(ctypes.POINTER(ctypes.POINTER(_U64))), ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int]),
    "svtgpu_cdef_controls_for_level": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(CdefControls)]),
    "svtgpu_cdef_state_create": (ctypes.c_int, [_P, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_cdef_state_destroy": (None, [_P]),
    "svtgpu_cdef_state_nfb": (_I32, [_P]),
    "svtgpu_cdef_set_block_mask": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_set_fb_bsize": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_search_frame": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(CdefControls), _I32, _P]),
    "svtgpu_cdef_pick": (ctypes.c_int, [_P, ctypes.POINTER(CdefControls), _I32, _U64, ctypes.POINTER(CdefParams),
                                        _P, _P]),
    "svtgpu_cdef_set_fb_strength": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_apply_frame": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(CdefParams), _P]),
    "svtgpu_cdef_pick_async": (ctypes.c_int, [_P, ctypes.POINTER(CdefControls), _I32, _U64, _P]),
    "svtgpu_cdef_read_params": (ctypes.c_int, [_P, ctypes.POINTER(CdefParams), _P, _P]),
    "svtgpu_cdef_set_fb_rows": (ctypes.c_int, [_P, _I32, _I32]),
    "svtgpu_cdef_bind_tables": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_bind_dir_tables": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_cdef_clear_tables": (ctypes.c_int, [_P, _P]),
    "svtgpu_cdef_read_state": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "svtgpu_cdef_mse_device_ptr": (_P, [_P]),
    **{"svtgpu_lpf_%s_%d" % (d, n): _LPF8 for d in ("horizontal", "vertical") for n in (4, 6, 8, 14)},
    **{"svtgpu_highbd_lpf_%s_%d" % (d, n): _LPF16 for d in ("horizontal", "vertical") for n in (4, 6, 8, 14)},
    "svtgpu_dlf_state_create": (ctypes.c_int, [_P, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_dlf_state_destroy": (None, [_P]),
    "svtgpu_dlf_set_mode_info": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_dlf_set_mode_info_device": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_dlf_frame": (ctypes.c_int, [_P, _P, ctypes.POINTER(LfParams), _I32, _I32, _P]),
    "svtgpu_dlf_frame_to": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LfParams), _I32, _I32, _P]),
    "svtgpu_dlf_pick": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LfParams), _I32, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_dlf_pick_async": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LfParams), _I32, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_dlf_read_levels": (ctypes.c_int, [_P, ctypes.POINTER(LfParams), _P]),
    "svtgpu_dlf_async_rounds": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_dlf_pick_by_q": (ctypes.c_int, [_P, _P]),
    "svtgpu_dlf_qp_based_param": (ctypes.c_int, [_I32, _I32, _I32, _P, _P]),
    "svtgpu_plane_sse": (ctypes.c_int, [_P, _P, _I32, ctypes.POINTER(_U64), _P]),
    **{"svtgpu_aom_sad%dx%d" % s: (ctypes.c_uint32, [_P, ctypes.c_int, _P, ctypes.c_int]) for s in MD_SIZES},
    **{"svtgpu_aom_sad%dx%dx4d" % s: (None, [_P, ctypes.c_int, _P, ctypes.c_int, _P]) for s in MD_SIZES},
    **{"svtgpu_aom_variance%dx%d" % s: (ctypes.c_uint32, [_P, ctypes.c_int, _P, ctypes.c_int,
                                                          ctypes.POINTER(ctypes.c_uint32)]) for s in MD_SIZES},
    **{"svtgpu_aom_highbd_10_variance%dx%d" % s: (ctypes.c_uint32, [_P, ctypes.c_int, _P, ctypes.c_int,
                                                                    ctypes.POINTER(ctypes.c_uint32)])
       for s in MD_SIZES},
    "svtgpu_sad_16b_kernel": (ctypes.c_uint32, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32]),
    "svtgpu_aom_sse": (ctypes.c_int64, [_P, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "svtgpu_aom_highbd_sse": (ctypes.c_int64, [_P, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "svtgpu_spatial_full_distortion_kernel": (_U64, [_P, ctypes.c_uint32, ctypes.c_uint32, _P, ctypes.c_int32,
                                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "svtgpu_full_distortion_kernel16_bits": (_U64, [_P, ctypes.c_uint32, ctypes.c_uint32, _P, ctypes.c_int32,
                                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "svtgpu_nxm_sad_kernel": (ctypes.c_uint32, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_uint32]),
    "svtgpu_nxm_sad_kernel_sub_sampled": (ctypes.c_uint32, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32,
                                                            ctypes.c_uint32]),
    "svtgpu_aom_mse16x16": (ctypes.c_uint32, [_P, _I32, _P, _I32, ctypes.POINTER(ctypes.c_uint32)]),
    "svtgpu_aom_highbd_8_mse16x16": (None, [_P, _I32, _P, _I32, ctypes.POINTER(ctypes.c_uint32)]),
    "svtgpu_aom_variance_highbd": (ctypes.c_uint32, [_P, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_uint32)]),
    **{"svtgpu_aom_sub_pixel_variance%dx%d" % s: (ctypes.c_uint32, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P,
                                                                    ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)])
       for s in MD_SIZES},
    "svtgpu_cdef_filter_block_8xn_16": (None, [_P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _I32, ctypes.c_uint8,
                                               ctypes.c_uint8]),
    "svtgpu_aom_copy_rect8_8bit_to_16bit": (None, [_P, _I32, _P, _I32, _I32, _I32]),
    "svtgpu_av1_compute_stats": (None, [_I32, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P]),
    "svtgpu_av1_compute_stats_highbd": (None, [_I32, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _I32]),
    "svtgpu_av1_lowbd_pixel_proj_error": (ctypes.c_int64, [_P, _I32, _I32, _I32, _P, _I32, _P, _I32, _P, _I32, _P, _P]),
    "svtgpu_av1_highbd_pixel_proj_error": (ctypes.c_int64, [_P, _I32, _I32, _I32, _P, _I32, _P, _I32, _P, _I32, _P,
                                                            _P]),
    "svtgpu_get_proj_subspace": (None, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int,
                                        _P, ctypes.c_int, _P, ctypes.c_int, _P, _P]),
    "svtgpu_md_batch_create": (ctypes.c_int, [_P, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_me_batch_create": (ctypes.c_int, [_P, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_convert_8bit_to_16bit": (None, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "svtgpu_convert_16bit_to_8bit": (None, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "svtgpu_aom_generate_padding": (None, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32]),
    "svtgpu_aom_generate_padding16_bit": (None, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_uint32]),
    "svtgpu_extend_frame": (None, [_P, _I32, _I32, _I32, _I32, _I32, _I32]),
    "svtgpu_convert_plane": (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_pad_plane": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_extend_plane": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_frame_convert": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_me_batch_destroy": (None, [_P]),
    "svtgpu_me_set_origins": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_me_search": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_me_read": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P]),
    "svtgpu_ext_all_sad_calculation_8x8_16x16": (None, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32, _P,
                                                        _P, _P, _P, _P, _P, ctypes.c_uint8]),
    "svtgpu_ext_eight_sad_calculation_32x32_64x64": (None, [_P, _P, _P, _P, _P, ctypes.c_uint32, _P]),
    "svtgpu_ext_sad_calculation_8x8_16x16": (None, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, _P, _P, _P, _P,
                                                    ctypes.c_uint32, _P, _P, ctypes.c_uint8]),
    "svtgpu_ext_sad_calculation_32x32_64x64": (None, [_P, _P, _P, _P, _P, ctypes.c_uint32, _P]),
    "svtgpu_sad_loop_kernel": (None, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _P,
                                      _P, _P, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_int16, ctypes.c_int16]),
    "svtgpu_pme_sad_loop_kernel": (None, [_P, _P, ctypes.c_uint32, _P, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, _P, _P, _P, ctypes.c_int16, ctypes.c_int16, ctypes.c_int16,
                                          ctypes.c_int16, ctypes.c_int16, ctypes.c_int16, ctypes.c_int16]),
    "svtgpu_md_batch_destroy": (None, [_P]),
    "svtgpu_md_batch_nsb": (_I32, [_P]),
    "svtgpu_md_set_mvs": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_md_dist_batch": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P]),
    "svtgpu_md_read": (ctypes.c_int, [_P, _P, _I32, _I32, _P]),
    "svtgpu_md_out_device_ptr": (_P, [_P]),
    "svtgpu_md_moments_device_ptr": (_P, [_P]),
    "svtgpu_md_expand": (ctypes.c_int, [_P, _I32, _I32, _P]),
    "svtgpu_md_layout": (None, [_P, _P, _P]),
    "svtgpu_av1_wiener_convolve_add_src": (None, [_P, ctypes.c_ssize_t, _P, ctypes.c_ssize_t, _P, _P, _I32, _I32,
                                                  ctypes.POINTER(ConvolveParams)]),
    "svtgpu_av1_highbd_wiener_convolve_add_src": (None, [_P, ctypes.c_ssize_t, _P, ctypes.c_ssize_t, _P, _P, _I32,
                                                         _I32, ctypes.POINTER(ConvolveParams), _I32]),
    "svtgpu_av1_selfguided_restoration": (None, [_P, _I32, _I32, _I32, _P, _P, _I32, _I32, _I32, _I32]),
    "svtgpu_apply_selfguided_restoration": (None, [_P, _I32, _I32, _I32, _I32, _P, _P, _I32, _P, _I32, _I32]),
    "svtgpu_lr_state_create": (ctypes.c_int, [_P, _I32, _I32, _P, ctypes.POINTER(_P)]),
    "svtgpu_lr_state_destroy": (None, [_P]),
    "svtgpu_lr_units": (ctypes.c_int, [_P, _I32, ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "svtgpu_lr_set_units": (ctypes.c_int, [_P, _I32, _P, _P]),
    "svtgpu_lr_apply_frame": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "svtgpu_lr_search_frame": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LrSearchControls), _P, _P, _P]),
    "svtgpu_lr_controls_for_level": (ctypes.c_int, [_I32, _I32, ctypes.POINTER(LrSearchControls)]),
    "svtgpu_lr_search_units": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LrSearchControls), _P, _P, _P, _P]),
    "svtgpu_lr_finish_plane": (ctypes.c_int, [ctypes.POINTER(LrSearchControls), _I32, _I32, _P, _P, _P]),
    "svtgpu_lr_finish_frame": (ctypes.c_int, [ctypes.POINTER(LrSearchControls), _P, _P, _P, _P]),
    "svtgpu_lr_search_frame_async": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(LrSearchControls), _P]),
    "svtgpu_lr_read_result": (ctypes.c_int, [_P, _P, _P]),
    "svtgpu_lr_read_units": (ctypes.c_int, [_P, _I32, _P, _P]),
    "svtgpu_lr_profile": (ctypes.c_int, [_P, _I32, _P]),
    "svtgpu_transfer_bytes": (ctypes.c_int, [_P, _P, _I32]),
    "svtgpu_comm_unique_id": (ctypes.c_int, [_P]),
    "svtgpu_comm_create": (ctypes.c_int, [_P, _I32, _I32, _P, ctypes.POINTER(_P)]),
    "svtgpu_comm_create_bounded": (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_comm_create_host": (ctypes.c_int, [_I32, _I32, _P, ctypes.POINTER(_P)]),
    "svtgpu_comm_destroy": (None, [_P]),
    "svtgpu_comm_nranks": (_I32, [_P]),
    "svtgpu_comm_rank": (_I32, [_P]),
    "svtgpu_comm_allreduce_u64": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _I32, _P]),
    "svtgpu_comm_set_timeout": (ctypes.c_int, [_P, _I32]),
    "svtgpu_comm_timeout_ms": (_I32, [_P]),
    "svtgpu_comm_set_slot": (ctypes.c_int, [_P, _I32]),
    "svtgpu_comm_failed": (_I32, [_P]),
    "svtgpu_comm_sync": (ctypes.c_int, [_P, _P]),
    "svtgpu_debug_stall": (ctypes.c_int, [_P, _P, _I32]),
    "svtgpu_shim_calls": (ctypes.c_uint64, []),
    "svtgpu_tile_plan": (ctypes.c_int, [_I32, _I32, _P, _I32, _I32, _I32, _P]),
    "svtgpu_tile_plan_sb": (ctypes.c_int, [_I32, _I32, _P, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_tile_plan_crop": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _I32, _I32, _I32, _I32, _P]),
    "svtgpu_dlf_set_tile": (ctypes.c_int, [_P, _P, _P, _P]),
    "svtgpu_dlf_set_crop": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32]),
    "svtgpu_cdef_set_tile": (ctypes.c_int, [_P, _P, _P, _P]),
    "svtgpu_lr_set_tile": (ctypes.c_int, [_P, _P, _P, _P]),
    "svtgpu_buffer_alloc": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(_P)]),
    "svtgpu_buffer_free": (None, [_P]),
    "svtgpu_buffer_upload": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _P]),
    "svtgpu_buffer_download": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _P]),
    "svtgpu_ccso_grid": (ctypes.c_int, [_I32, _I32, _I32, ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "svtgpu_ccso_extend_luma": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P]),
    "svtgpu_ccso_state_create": (ctypes.c_int, [_P, _I32, _I32, ctypes.POINTER(_P)]),
    "svtgpu_ccso_state_destroy": (None, [_P]),
    "svtgpu_ccso_search_plane": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, ctypes.POINTER(CcsoParams), _P,
                                                _P]),
    "svtgpu_ccso_search_frame": (ctypes.c_int, [_P, _P, _P * 3, _P * 3, _I32, _I32, _I32, ctypes.POINTER(CcsoParams),
                                                _P, ctypes.POINTER(_I32), _P]),
    "svtgpu_ccso_apply_plane": (ctypes.c_int, [_P, _P, _I32, _I32, _P, _I32, _I32, ctypes.POINTER(CcsoParams), _P,
                                               _P]),
    "svtgpu_compute_distortion_block": (ctypes.c_uint64, [_P, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "svtgpu_ccso_derive_src_block": (None, [_P, _P, _P] + [ctypes.c_int] * 10 + [_P, ctypes.c_int, ctypes.c_int]),
    "svtgpu_ccso_filter_block_hbd_with_buf": (None, [_P, _P, _P, _P] + [ctypes.c_int] * 7 + [_P] +
                                              [ctypes.c_int] * 4 + [ctypes.c_uint8, ctypes.c_uint8]),
    "svtgpu_ccso_filter_block_hbd_wo_buf": (None, [_P, _P] + [ctypes.c_int] * 4 + [_P, _P] + [ctypes.c_int] * 6 +
                                            [_P, ctypes.c_int, ctypes.c_int, ctypes.c_bool, ctypes.c_uint8,
                                             ctypes.c_int, ctypes.c_uint8]),
}

_lib = None


def lib():
    """Load libsvtgpu.so (in-tree build).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libsvtgpu.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class SvtGpuError(RuntimeError):
    pass


def check(rc):
    if rc != SVTGPU_OK:
        raise SvtGpuError("svtgpu error %d: %s" % (rc, lib().svtgpu_error_string(rc).decode()))
    return rc


def require_device():
    if not lib().svtgpu_device_available():
        raise SvtGpuError("no gfx950 device visible: the HIP path is required (no CPU fallback)")


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Context:
    def __init__(self, device=0):
        require_device()
        h = _P()
        check(lib().svtgpu_context_create(device, ctypes.byref(h)))
        self.h = h

    @property
    def stream(self):
        return lib().svtgpu_context_stream(self.h)

    def synchronize(self, stream=None):
        check(lib().svtgpu_synchronize(self.h, stream))

    def stream_create(self, priority=0):
        """A new hipStream_t (as an int) for the frame-level calls: one hardware queue each while the process has no
        more streams than GPU_MAX_HW_QUEUES (svtgpu_stream_create).  Wrap it with torch.cuda.ExternalStream to time
        it with torch events; destroy it with stream_destroy."""
        h = _P()
        check(lib().svtgpu_stream_create(self.h, int(priority), ctypes.byref(h)))
        return h.value

    @staticmethod
    def stream_destroy(stream):
        lib().svtgpu_stream_destroy(stream)

    def debug_stall(self, ms, stream=None):
        """Test support: hold `stream` busy for `ms` milliseconds (one spinning wave)."""
        check(lib().svtgpu_debug_stall(self.h, stream, int(ms)))

    def close(self):
        if self.h:
            lib().svtgpu_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Frame:
    """Device-resident 4:2:0 picture (uint8 for 8-bit, uint16 for 10-bit samples)."""

    def __init__(self, ctx, width, height, bit_depth):
        self.ctx, self.width, self.height, self.bit_depth = ctx, width, height, bit_depth
        self.dtype = np.uint16 if bit_depth > 8 else np.uint8
        h = _P()
        check(lib().svtgpu_frame_create(ctx.h, width, height, bit_depth, ctypes.byref(h)))
        self.h = h

    def plane_shape(self, p):
        return (self.height, self.width) if p == 0 else (self.height // 2, self.width // 2)

    def upload(self, planes, stream=None, rect=None):
        """All samples, or (rect = luma {x0, y0, x1, y1}) only those of the rectangle: chroma halved, rounded outward
        (svtgpu_frame_upload_rect; a rank of a tiled picture uploads its plan's in_rect)."""
        keep = []
        for p, a in enumerate(planes):
            a = np.ascontiguousarray(a, dtype=self.dtype)
            assert a.shape == self.plane_shape(p), (a.shape, self.plane_shape(p))
            keep.append(a)
            if rect is None:
                check(lib().svtgpu_frame_upload(self.h, p, ptr(a), a.shape[1], stream))
            else:
                r = chroma_rect(rect, a.shape) if p else [int(v) for v in rect]
                check(lib().svtgpu_frame_upload_rect(self.h, p, ptr(a), a.shape[1], _rect(r), stream))
        self.ctx.synchronize(stream)  # host buffers must outlive the copies

    def download(self, stream=None):
        out = []
        for p in range(3):
            a = np.empty(self.plane_shape(p), dtype=self.dtype)
            check(lib().svtgpu_frame_download(self.h, p, ptr(a), a.shape[1], stream))
            out.append(a)
        return out

    def close(self):
        if self.h:
            lib().svtgpu_frame_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cdef_controls(level):
    c = CdefControls()
    check(lib().svtgpu_cdef_controls_for_level(level, ctypes.byref(c)))
    return c


class TilePlan(ctypes.Structure):
    """SvtGpuTilePlan: what one rank of a picture tiled over GPUs computes (svtgpu_tile_plan)."""
    _fields_ = [("tile", _I32 * 4), ("fb_rect", _I32 * 4), ("lr_units", (_I32 * 4) * 3), ("lr_out", (_I32 * 4) * 3),
                ("cdef_out", _I32 * 4), ("dlf_out", _I32 * 4), ("in_rect", _I32 * 4)]

    def rects(self):
        return {k: (np.array(getattr(self, k)).tolist()) for k, _ in self._fields_}


def chroma_rect(r, shape):
    """A luma rectangle {x0, y0, x1, y1} on a 4:2:0 chroma plane of `shape` (rows, cols): halved, rounded outward."""
    return [int(r[0]) // 2, int(r[1]) // 2, min(shape[1], (int(r[2]) + 1) // 2), min(shape[0], (int(r[3]) + 1) // 2)]


def tile_grid(n):
    """gx x gy of n ranks: the widest split with gx <= gy (1x1, 1x2, 2x2, 2x4 for 1, 2, 4, 8 GPUs)."""
    gx = max(d for d in range(1, int(n ** 0.5) + 1) if n % d == 0)
    return gx, n // gx


def tile_plan(width, height, unit_size, gx, gy, rank, sb=64, crop=None):
    """svtgpu_tile_plan_sb; crop=(w, h): a picture whose crop size is below the 8-aligned coded size width x height
    (svtgpu_tile_plan_crop)."""
    us = np.ascontiguousarray(unit_size, np.int32)
    t = TilePlan()
    if crop is None:
        check(lib().svtgpu_tile_plan_sb(width, height, ptr(us), sb, gx, gy, rank, ctypes.byref(t)))
    else:
        check(lib().svtgpu_tile_plan_crop(width, height, int(crop[0]), int(crop[1]), ptr(us), sb, gx, gy, rank,
                                          ctypes.byref(t)))
    return t


_ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t)


class _HostTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allreduce_u64", _ALLREDUCE_FN)]


class Comm:
    """SvtGpuComm: the ranks of a picture tiled over GPUs.  Comm.rccl: RCCL over xGMI (one rank per device; rank 0
    makes the id with unique_id(), the caller broadcasts it); Comm.host: a host transport, `fn(words)` summing a uint64
    numpy array over the ranks in place (e.g. a gloo all_reduce) — several ranks on one GPU, CPU rehearsals.  Every
    exchange is bounded by `timeout_ms` (a host transport bounds its own wait by it: `fn(words, timeout_ms)` when fn
    takes two arguments, raising on expiry); an expired exchange raises SvtGpuError naming it, and the communicator
    fails from then on (`failed`)."""

    def __init__(self, h, keep=None):
        self.h, self._keep = h, keep

    @staticmethod
    def unique_id():
        b = (ctypes.c_uint8 * 128)()
        check(lib().svtgpu_comm_unique_id(b))
        return bytes(b)

    @classmethod
    def rccl(cls, ctx, nranks, rank, uid, timeout_ms=0, slot=-1):
        """svtgpu_comm_create_bounded: the RCCL communicator, its init bounded by timeout_ms (0: the default
        deadline); a peer that never joins raises SvtGpuError naming "communicator init", the slot and the rank."""
        b = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = _P()
        check(lib().svtgpu_comm_create_bounded(ctx.h, nranks, rank, b, int(timeout_ms), int(slot), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def host(cls, nranks, rank, fn):
        import inspect
        two = len(inspect.signature(fn).parameters) >= 2
        box = []  # the Comm, for its deadline

        def cb(user, buf, n):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                if two:
                    fn(a, box[0]().timeout_ms)
                else:
                    fn(a)
                return 0
            except Exception:  # reported through the library's return code
                import traceback
                traceback.print_exc()
                return -1
        f = _ALLREDUCE_FN(cb)
        t = _HostTransport(None, f)
        h = _P()
        check(lib().svtgpu_comm_create_host(nranks, rank, ctypes.byref(t), ctypes.byref(h)))
        c = cls(h, keep=(f, t))
        import weakref
        box.append(weakref.ref(c))  # no reference cycle through the callback
        return c

    @property
    def nranks(self):
        return lib().svtgpu_comm_nranks(self.h)

    @property
    def timeout_ms(self):
        return lib().svtgpu_comm_timeout_ms(self.h)

    def set_timeout(self, ms):
        check(lib().svtgpu_comm_set_timeout(self.h, int(ms)))

    def set_slot(self, slot):
        check(lib().svtgpu_comm_set_slot(self.h, int(slot)))

    @property
    def failed(self):
        return bool(lib().svtgpu_comm_failed(self.h))

    def sync(self, stream=None):
        """Wait for `stream`, bounded by the deadline while a device-side exchange is outstanding."""
        check(lib().svtgpu_comm_sync(self.h, stream))

    def allreduce(self, words, stream=None):
        """Sum a host uint64 array over the ranks in place."""
        a = np.ascontiguousarray(words, np.uint64)
        check(lib().svtgpu_comm_allreduce_u64(self.h, ptr(a), a.size, 0, stream))
        return a

    def allreduce_device(self, dev_ptr, n, stream=None):
        """Sum n uint64 words of device memory over the ranks in place (enqueued on `stream`)."""
        check(lib().svtgpu_comm_allreduce_u64(self.h, ctypes.c_void_p(dev_ptr), n, 1, stream))

    def close(self):
        if self.h:
            lib().svtgpu_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _rect(r):
    return None if r is None else (_I32 * 4)(*[int(x) for x in r])


def _rects3(r):
    return None if r is None else ((_I32 * 4) * 3)(*[(_I32 * 4)(*[int(x) for x in q]) for q in r])


class CdefState:
    """Device search state of one frame (mse_seg / skip_cdef_seg / cdef_dir_data)."""

    def __init__(self, ctx, width, height):
        self.ctx, self.width, self.height = ctx, width, height
        h = _P()
        check(lib().svtgpu_cdef_state_create(ctx.h, width, height, ctypes.byref(h)))
        self.h = h
        self.nfb = lib().svtgpu_cdef_state_nfb(h)

    def set_block_mask(self, mask, stream=None):
        if mask is None:
            check(lib().svtgpu_cdef_set_block_mask(self.h, None, stream))
        else:
            self._mask = np.ascontiguousarray(mask, dtype=np.uint8)
            check(lib().svtgpu_cdef_set_block_mask(self.h, ptr(self._mask), stream))

    def set_fb_bsize(self, fb_bsize, stream=None):
        """SB128 mode info: BlockSize at each 64x64 filter block's top-left (None = SB64)."""
        if fb_bsize is None:
            check(lib().svtgpu_cdef_set_fb_bsize(self.h, None, stream))
        else:
            self._fbb = np.ascontiguousarray(fb_bsize, dtype=np.uint8)
            assert self._fbb.size == self.nfb
            check(lib().svtgpu_cdef_set_fb_bsize(self.h, ptr(self._fbb), stream))

    def search(self, recon, source, ctrls, base_q_idx, stream=None):
        check(lib().svtgpu_cdef_search_frame(self.h, recon.h, source.h, ctypes.byref(ctrls), base_q_idx, stream))

    def pick(self, ctrls, base_q_idx, lam, stream=None):
        prm = CdefParams()
        fbs = np.zeros(self.nfb, dtype=np.int8)
        check(lib().svtgpu_cdef_pick(self.h, ctypes.byref(ctrls), base_q_idx, lam, ctypes.byref(prm), ptr(fbs), stream))
        return prm, fbs

    def pick_async(self, ctrls, base_q_idx, lam, stream=None):
        """svtgpu_cdef_pick_async: the pick in stream order, no host wait; apply(params=None) uses its result."""
        check(lib().svtgpu_cdef_pick_async(self.h, ctypes.byref(ctrls), base_q_idx, lam, stream))

    def read_params(self, stream=None):
        """The last pick_async's parameters and per-FB strength indices (waits for `stream`)."""
        prm = CdefParams()
        fbs = np.zeros(self.nfb, dtype=np.int8)
        check(lib().svtgpu_cdef_read_params(self.h, ctypes.byref(prm), ptr(fbs), stream))
        return prm, fbs

    def set_fb_strength(self, fbs, stream=None):
        self._fbs = np.ascontiguousarray(fbs, dtype=np.int8)
        check(lib().svtgpu_cdef_set_fb_strength(self.h, ptr(self._fbs), stream))

    def apply(self, recon, out, params, stream=None):
        """params None: the last pick_async's parameters, from device memory."""
        check(lib().svtgpu_cdef_apply_frame(self.h, recon.h, out.h, ctypes.byref(params) if params is not None else None,
                                            stream))

    def read(self, stream=None):
        mse = np.empty((2, self.nfb, 64), dtype=np.uint64)
        skip = np.empty(self.nfb, dtype=np.uint8)
        d = np.empty((self.nfb, 64), dtype=np.uint8)
        v = np.empty((self.nfb, 64), dtype=np.int32)
        check(lib().svtgpu_cdef_read_state(self.h, ptr(mse), ptr(skip), ptr(d), ptr(v), stream))
        return mse, skip, d, v

    def set_fb_rows(self, begin, end):
        check(lib().svtgpu_cdef_set_fb_rows(self.h, begin, end))

    def set_tile(self, fb_rect=None, out_rect=None, comm=None):
        """svtgpu_cdef_set_tile: search fb_rect, pick over the tables summed over `comm`, apply into out_rect."""
        check(lib().svtgpu_cdef_set_tile(self.h, _rect(fb_rect), _rect(out_rect), comm.h if comm else None))

    def bind_tables(self, mse_dev_ptr, skip_dev_ptr):
        check(lib().svtgpu_cdef_bind_tables(self.h, mse_dev_ptr, skip_dev_ptr))

    def bind_dir_tables(self, dir_dev_ptr, var_dev_ptr):
        check(lib().svtgpu_cdef_bind_dir_tables(self.h, dir_dev_ptr, var_dev_ptr))

    def clear_tables(self, stream=None):
        check(lib().svtgpu_cdef_clear_tables(self.h, stream))

    def mse_device_ptr(self):
        return lib().svtgpu_cdef_mse_device_ptr(self.h)

    def close(self):
        if self.h:
            lib().svtgpu_cdef_state_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DlfState:
    """Deblocking state of one picture size: the device mode-info grid and the level tables."""

    def __init__(self, ctx, width, height):
        self.ctx, self.width, self.height = ctx, width, height
        self.mi_rows, self.mi_cols = ((height + 7) & ~7) >> 2, ((width + 7) & ~7) >> 2
        h = _P()
        check(lib().svtgpu_dlf_state_create(ctx.h, width, height, ctypes.byref(h)))
        self.h = h

    def set_mode_info(self, mi, stream=None):
        """mi: structured array (LF_MI_DTYPE) or uint8 [mi_rows, mi_cols, 8]."""
        a = np.ascontiguousarray(mi)
        if a.dtype != LF_MI_DTYPE:
            a = np.ascontiguousarray(a.astype(np.uint8).reshape(self.mi_rows, self.mi_cols, 8))
        assert a.nbytes == self.mi_rows * self.mi_cols * 8, (a.shape, self.mi_rows, self.mi_cols)
        check(lib().svtgpu_dlf_set_mode_info(self.h, ptr(a), stream))  # staged: `mi` is free on return

    def set_mode_info_device(self, d_mi, stream=None):
        """The grid from device memory: a CUDA tensor of mi_rows * mi_cols * 8 bytes (or its address)."""
        if hasattr(d_mi, "data_ptr"):
            assert d_mi.is_cuda and d_mi.is_contiguous() and d_mi.numel() * d_mi.element_size() == \
                self.mi_rows * self.mi_cols * 8, (d_mi.shape, self.mi_rows, self.mi_cols)
            d_mi = d_mi.data_ptr()
        check(lib().svtgpu_dlf_set_mode_info_device(self.h, _P(d_mi), stream))

    def filter(self, frame, params, plane_start=0, plane_end=3, stream=None):
        """svtgpu_dlf_frame; params None: the levels of the last pick_async (on the device, in stream order)."""
        check(lib().svtgpu_dlf_frame(self.h, frame.h, None if params is None else ctypes.byref(params), plane_start,
                                     plane_end, stream))

    def filter_to(self, src, out, params, plane_start=0, plane_end=3, stream=None):
        """svtgpu_dlf_frame_to; params None: the levels of the last pick_async (on the device, in stream order)."""
        check(lib().svtgpu_dlf_frame_to(self.h, src.h, out.h, None if params is None else ctypes.byref(params),
                                        plane_start, plane_end, stream))

    def pick_async(self, recon, source, params, dlf_avg=0, dlf_avg_uv=0, temporal_layer_index=0, early_exit=2,
                   only_4x4=0, stream=None):
        """svtgpu_dlf_pick_async: the level search on the device, no host wait; filter(_to)(..., None) applies the
        picked levels, read_levels() returns them."""
        p = LfParams()
        ctypes.pointer(p)[0] = params
        check(lib().svtgpu_dlf_pick_async(self.h, recon.h, source.h, ctypes.byref(p), dlf_avg, dlf_avg_uv,
                                          temporal_layer_index, early_exit, only_4x4, stream))

    def async_rounds(self):
        """svtgpu_dlf_async_rounds: (rounds the last collected asynchronous search took, rounds enqueued)."""
        t, e = _I32(), _I32()
        check(lib().svtgpu_dlf_async_rounds(self.h, ctypes.byref(t), ctypes.byref(e)))
        return t.value, e.value

    def read_levels(self, stream=None):
        """svtgpu_dlf_read_levels: waits for the last pick_async and returns its LfParams."""
        p = LfParams()
        check(lib().svtgpu_dlf_read_levels(self.h, ctypes.byref(p), stream))
        return p

    def set_crop(self, crop_width, crop_height):
        """svtgpu_dlf_set_crop: no edge at or past the unpadded size is filtered (next set_mode_info on)."""
        check(lib().svtgpu_dlf_set_crop(self.h, crop_width, crop_height))

    def set_tile(self, sse_rect=None, out_rect=None, comm=None):
        """svtgpu_dlf_set_tile: trial SSEs over sse_rect summed over `comm`; the filter writes out_rect."""
        check(lib().svtgpu_dlf_set_tile(self.h, _rect(sse_rect), _rect(out_rect), comm.h if comm else None))

    def pick(self, recon, source, params, dlf_avg=0, dlf_avg_uv=0, temporal_layer_index=0, early_exit=2,
             only_4x4=0, stream=None):
        """Level search; `params` carries the previous levels in; returns the picked LfParams."""
        p = LfParams()
        ctypes.pointer(p)[0] = params
        check(lib().svtgpu_dlf_pick(self.h, recon.h, source.h, ctypes.byref(p), dlf_avg, dlf_avg_uv,
                                    temporal_layer_index, early_exit, only_4x4, stream))
        return p

    def close(self):
        if self.h:
            lib().svtgpu_dlf_state_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MeBatch:
    """Open-loop full-pel ME (svtgpu_me_search): every 64x64 block x reference over a search area; per (block,
    reference) the 85 best SADs / MVs in the reference's Z-order numbering (64 8x8, 16 16x16, 4 32x32, 1 64x64)."""

    def __init__(self, ctx, width, height, nref):
        self.ctx, self.width, self.height, self.nref = ctx, width, height, nref
        h = _P()
        check(lib().svtgpu_me_batch_create(ctx.h, width, height, nref, ctypes.byref(h)))
        self.h = h
        self.nsb = ((width + 63) // 64) * ((height + 63) // 64)

    def set_origins(self, origin, stream=None):
        a = np.ascontiguousarray(origin, dtype=np.int16)
        assert a.shape == (self.nsb, self.nref, 2), a.shape
        check(lib().svtgpu_me_set_origins(self.h, ptr(a), stream))

    def search(self, source, refs, saw, sah, sub=0, sb_begin=0, sb_end=None, stream=None):
        assert len(refs) == self.nref
        arr = (_P * self.nref)(*[r.h for r in refs])
        end = self.nsb if sb_end is None else sb_end
        check(lib().svtgpu_me_search(self.h, source.h, arr, saw, sah, int(sub), sb_begin, end, stream))

    def read(self, sb_begin=0, sb_end=None, stream=None):
        end = self.nsb if sb_end is None else sb_end
        sad = np.empty((end - sb_begin, self.nref, 85), np.uint32)
        mv = np.empty((end - sb_begin, self.nref, 85), np.uint32)
        check(lib().svtgpu_me_read(self.h, ptr(sad), ptr(mv), sb_begin, end, stream))
        return sad, mv

    def close(self):
        if self.h:
            lib().svtgpu_me_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MdBatch:
    """Batched MD distortion: every SB x reference x AV1 block shape (SAD, sse, variance)."""

    def __init__(self, ctx, width, height, nref):
        self.ctx, self.width, self.height, self.nref = ctx, width, height, nref
        h = _P()
        check(lib().svtgpu_md_batch_create(ctx.h, width, height, nref, ctypes.byref(h)))
        self.h = h
        self.nsb = lib().svtgpu_md_batch_nsb(h)

    def set_mvs(self, mv, stream=None):
        a = np.ascontiguousarray(mv, dtype=np.int16)
        assert a.shape == (self.nsb, self.nref, 2), a.shape
        check(lib().svtgpu_md_set_mvs(self.h, ptr(a), stream))

    def run(self, source, refs, sb_begin=0, sb_end=None, stream=None):
        assert len(refs) == self.nref
        arr = (_P * self.nref)(*[r.h for r in refs])
        end = self.nsb if sb_end is None else sb_end
        check(lib().svtgpu_md_dist_batch(self.h, source.h, arr, sb_begin, end, stream))

    def read(self, sb_begin=0, sb_end=None, stream=None):
        end = self.nsb if sb_end is None else sb_end
        out = np.empty((end - sb_begin, self.nref, 3, MD_BLOCKS), np.uint32)
        check(lib().svtgpu_md_read(self.h, ptr(out), sb_begin, end, stream))
        return out

    def expand(self, sb_begin=0, sb_end=None, stream=None):
        """svtgpu_md_expand: every shape's values of the SB range from the cell moments (in stream order)."""
        end = self.nsb if sb_end is None else sb_end
        check(lib().svtgpu_md_expand(self.h, sb_begin, end, stream))

    def out_device_ptr(self):
        return lib().svtgpu_md_out_device_ptr(self.h)

    def close(self):
        if self.h:
            lib().svtgpu_md_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def md_layout():
    w, h, o = (np.zeros(19, np.int32) for _ in range(3))
    lib().svtgpu_md_layout(ptr(w), ptr(h), ptr(o))
    return w, h, o


class LrState:
    """Loop-restoration state of one picture size: unit grid and per-unit parameters per plane."""

    def __init__(self, ctx, width, height, unit_size):
        self.ctx, self.width, self.height = ctx, width, height
        self.unit_size = list(unit_size)
        us = np.ascontiguousarray(unit_size, np.int32)
        h = _P()
        check(lib().svtgpu_lr_state_create(ctx.h, width, height, ptr(us), ctypes.byref(h)))
        self.h = h
        self.units = []
        for p in range(3):
            hu, vu = _I32(), _I32()
            check(lib().svtgpu_lr_units(h, p, ctypes.byref(hu), ctypes.byref(vu)))
            self.units.append((hu.value, vu.value))

    def set_units(self, plane, units, stream=None):
        u = np.ascontiguousarray(units, REST_UNIT_DTYPE)
        assert len(u) == self.units[plane][0] * self.units[plane][1], (len(u), self.units[plane])
        check(lib().svtgpu_lr_set_units(self.h, plane, ptr(u), stream))

    def search(self, recon, source, ctrls, stream=None, records=False):
        """svtgpu_lr_search_frame: picks frame types and unit parameters (kept on the device for apply).
        Returns the frame types and, with records=True, the per-unit search records."""
        ft = np.zeros(3, np.int32)
        recs = [np.zeros(hu * vu, LR_UNIT_SEARCH_DTYPE) for hu, vu in self.units] if records else None
        rp = (ctypes.c_void_p * 3)(*[r.ctypes.data for r in recs]) if records else None
        check(lib().svtgpu_lr_search_frame(self.h, recon.h, source.h, ctypes.byref(ctrls), ptr(ft), rp, stream))
        return ([int(x) for x in ft], recs) if records else [int(x) for x in ft]

    def search_async(self, recon, source, ctrls, stream=None):
        """svtgpu_lr_search_frame_async: search + device RD finish enqueued on `stream`, no host wait; apply(...,
        frame_type=None) applies the result in stream order, read_result() collects the frame types."""
        check(lib().svtgpu_lr_search_frame_async(self.h, recon.h, source.h, ctypes.byref(ctrls), stream))

    def read_units(self, plane, stream=None):
        """svtgpu_lr_read_units: the state's units of `plane` (waits for an asynchronous search)."""
        u = np.zeros(self.units[plane][0] * self.units[plane][1], REST_UNIT_DTYPE)
        check(lib().svtgpu_lr_read_units(self.h, plane, ptr(u), stream))
        return u

    def read_result(self, stream=None):
        """svtgpu_lr_read_result: waits for the last asynchronous search and returns its frame types."""
        ft = np.zeros(3, np.int32)
        check(lib().svtgpu_lr_read_result(self.h, ptr(ft), stream))
        return [int(x) for x in ft]

    def search_units(self, recon, source, ctrls, row_begin, row_end, records=None, stream=None):
        """svtgpu_lr_search_units: per-unit records of the unit rows [row_begin[p], row_end[p]) of every plane,
        written into `records` (per-plane arrays of all units; allocated zeroed when None).  No RD finish."""
        if records is None:
            records = [np.zeros(hu * vu, LR_UNIT_SEARCH_DTYPE) for hu, vu in self.units]
        rb = np.ascontiguousarray(row_begin, np.int32)
        re_ = np.ascontiguousarray(row_end, np.int32)
        rp = (ctypes.c_void_p * 3)(*[r.ctypes.data for r in records])
        check(lib().svtgpu_lr_search_units(self.h, recon.h, source.h, ctypes.byref(ctrls), ptr(rb), ptr(re_), rp,
                                           stream))
        return records

    PROFILE_CLASSES = ("stats", "sgr_filters", "wiener_trials", "projection", "other", "sgr_moments")

    def profile(self, enable=True, events=False, serial=False):
        """svtgpu_lr_profile: device-clock timing of the searches (enable: True = every class, a class name or a
        list of names = those classes, False = off).  Returns the per-class {launches, ms (device clock), ms_events
        (HIP events around each launch), bytes} totals of the
        searches timed since the previous call (kernel classes of svtgpu.h; untimed classes read 0) plus
        "searches", their count; reading synchronizes the device."""
        if enable is True:
            mask = -1
        elif not enable:
            mask = 0
        else:
            names = [enable] if isinstance(enable, str) else list(enable)
            mask = sum(1 << self.PROFILE_CLASSES.index(c) for c in names)
        if mask and events:
            mask = (63 if mask < 0 else mask) | 64
        if serial:  # both LR chains on one stream: each kernel's duration is its own (measurement)
            mask = (63 if mask < 0 else mask) | 128
        raw = np.zeros(1, LR_PROFILE_DTYPE)
        check(lib().svtgpu_lr_profile(self.h, mask, ptr(raw)))
        out = {c: {"launches": int(raw["launches"][0][i]), "ms": float(raw["ms"][0][i]),
                   "ms_events": float(raw["ms_events"][0][i]), "bytes": float(raw["bytes"][0][i])}
               for i, c in enumerate(self.PROFILE_CLASSES)}
        out["searches"] = int(raw["searches"][0])
        return out

    def set_tile(self, units=None, out=None, comm=None):
        """svtgpu_lr_set_tile: search units[p], records summed over `comm`, finish everywhere, apply into out[p]."""
        check(lib().svtgpu_lr_set_tile(self.h, _rects3(units), _rects3(out), comm.h if comm else None))

    def apply(self, deblocked, cdef_out, out, frame_type, stream=None):
        """svtgpu_lr_apply_frame; frame_type None: the units the last (asynchronous) search left on the device."""
        ft = None if frame_type is None else np.ascontiguousarray(frame_type, np.int32)
        check(lib().svtgpu_lr_apply_frame(self.h, deblocked.h, cdef_out.h, out.h, None if ft is None else ptr(ft),
                                          stream))

    def close(self):
        if self.h:
            lib().svtgpu_lr_state_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lr_controls(wn_level, sg_level, rdmult=0, switchable=(0, 0, 0), wiener=(0, 0), sgrproj=(0, 0)):
    """SvtGpuLrSearchControls of the reference's wn/sg filter levels plus the encoder's rate inputs."""
    c = LrSearchControls()
    check(lib().svtgpu_lr_controls_for_level(wn_level, sg_level, ctypes.byref(c)))
    c.rdmult = rdmult
    for i, v in enumerate(switchable):
        c.switchable_restore_cost[i] = v
    for i, v in enumerate(wiener):
        c.wiener_restore_cost[i] = v
    for i, v in enumerate(sgrproj):
        c.sgrproj_restore_cost[i] = v
    return c


def lr_finish_plane(ctrls, plane, records):
    """svtgpu_lr_finish_plane (host only): (frame restoration type, units) of a plane from all its records."""
    r = np.ascontiguousarray(records, LR_UNIT_SEARCH_DTYPE)
    units = np.zeros(len(r), REST_UNIT_DTYPE)
    ft = _I32()
    check(lib().svtgpu_lr_finish_plane(ctypes.byref(ctrls), plane, len(r), ptr(r), ctypes.byref(ft), ptr(units)))
    return ft.value, units


def lr_finish_frame(ctrls, records):
    """svtgpu_lr_finish_frame (host only): rest_finish_search of the whole frame over one RestUnitSearchInfo array
    shared by the planes.  records: per-plane arrays of all units.  Returns (frame types [3], units [3])."""
    rs = [np.ascontiguousarray(r, LR_UNIT_SEARCH_DTYPE) for r in records]
    units = [np.zeros(len(r), REST_UNIT_DTYPE) for r in rs]
    n = np.array([len(r) for r in rs], np.int32)
    ft = np.zeros(3, np.int32)
    rp = (ctypes.c_void_p * 3)(*[r.ctypes.data for r in rs])
    up = (ctypes.c_void_p * 3)(*[u.ctypes.data for u in units])
    check(lib().svtgpu_lr_finish_frame(ctypes.byref(ctrls), ptr(n), rp, ptr(ft), up))
    return [int(x) for x in ft], units


# ---------------------------------------------------------------------------------------------
# multi-GPU decomposition (one rank per GPU): balanced bands of rows; the only data-path exchanges are
# the CDEF mse/skip table all-reduce and the LR record all-gather
# ---------------------------------------------------------------------------------------------
def band(count, n, rank):
    """[begin, end) of `rank`'s share of `count` rows split into `n` balanced contiguous bands."""
    edges = np.linspace(0, count, n + 1).round().astype(int)
    return int(edges[rank]), int(edges[rank + 1])


def lr_unit_rows(units, n, rank):
    """Per-plane unit-row bands (row_begin[3], row_end[3]) of `rank` for an LrState.units list [(hu, vu)]."""
    rb, re_ = zip(*(band(vu, n, rank) for _, vu in units))
    return list(rb), list(re_)


def gather_lr_records(records, units, n, rank, group=None, device=None):
    """All-gather the per-unit LR search records of every rank's unit-row band (torch.distributed; RCCL with
    device="cuda", gloo with device=None).  `records`: per-plane arrays of all units with this rank's band
    filled.  Returns the merged per-plane arrays (every unit from the rank that searched it)."""
    import torch
    import torch.distributed as dist
    merged = []
    for p, (hu, vu) in enumerate(units):
        raw = torch.from_numpy(np.ascontiguousarray(records[p]).view(np.uint8).copy())
        if device is not None:
            raw = raw.to(device)
        parts = [torch.empty_like(raw) for _ in range(n)]
        dist.all_gather(parts, raw, group=group)
        out = np.zeros(hu * vu, LR_UNIT_SEARCH_DTYPE)
        for r in range(n):
            b, e = band(vu, n, r)
            got = parts[r].cpu().numpy().view(LR_UNIT_SEARCH_DTYPE)
            out[b * hu:e * hu] = got[b * hu:e * hu]
        merged.append(out)
    return merged


class CcsoState:
    """CCSO on the device: the reference's ccso_search / derive_ccso_filter and ccso_frame
    (EbPickccso.c:464-815, EbCcso.c:626-678) over device buffers given as integer addresses (e.g. a torch tensor's
    data_ptr()).  org / rec / the planes' samples use the luma width as stride (ccso_stride)."""

    def __init__(self, ctx, width, height):
        self.ctx, self.width, self.height = ctx, width, height
        h = _P()
        check(lib().svtgpu_ccso_state_create(ctx.h, width, height, ctypes.byref(h)))
        self.h = h

    def grid(self, plane):
        a, b = _I32(), _I32()
        check(lib().svtgpu_ccso_grid(self.width, self.height, plane, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def extend(self, luma, bits, stride, ext, stream=None):
        """ext_rec_y (EbPickccso.c:907-918 + extend_ccso_border) from a device luma plane into `ext`."""
        check(lib().svtgpu_ccso_extend_luma(luma, bits, stride, self.width, self.height, ext, stream))

    def search_plane(self, ext, org, rec, plane, bit_depth, rdmult, stream=None, read=True):
        """derive_ccso_filter of one plane; (CcsoParams, flags (nvfb, nhfb) uint8) when read, else None (the result
        stays on the device for apply(params=None))."""
        if not read:
            check(lib().svtgpu_ccso_search_plane(self.h, ext, org, rec, plane, bit_depth, rdmult, None, None, stream))
            return None
        prm, flags = CcsoParams(), np.zeros(self.grid(plane), np.uint8)
        check(lib().svtgpu_ccso_search_plane(self.h, ext, org, rec, plane, bit_depth, rdmult, ctypes.byref(prm),
                                             ptr(flags), stream))
        return prm, flags

    def search_frame(self, ext, org, rec, bit_depth, rdmult, base_q_idx, stream=None, read=True):
        """ccso_search: (rc, [CcsoParams] * 3, [flags] * 3, frame_flag); rc 1 = rdmult overflow, nothing searched.
        read=False: no read-back and no host wait (rc only); the results stay on the device for apply()."""
        if not read:
            rc = lib().svtgpu_ccso_search_frame(self.h, ext, (_P * 3)(*org), (_P * 3)(*rec), bit_depth, rdmult,
                                                base_q_idx, None, None, ctypes.byref(_I32(0)), stream)
            if rc not in (0, 1):
                check(rc)
            return rc
        prms = (CcsoParams * 3)()
        flags = [np.zeros(self.grid(p), np.uint8) for p in range(3)]
        ff = _I32(0)
        rc = lib().svtgpu_ccso_search_frame(self.h, ext, (_P * 3)(*org), (_P * 3)(*rec), bit_depth, rdmult,
                                            base_q_idx, prms, (_P * 3)(*[f.ctypes.data for f in flags]),
                                            ctypes.byref(ff), stream)
        if rc not in (0, 1):
            check(rc)
        return rc, list(prms), flags, ff.value

    def apply(self, ext, plane, bit_depth, dst, dst_bits, dst_stride, params=None, flags=None, stream=None):
        """ccso_frame's body for one plane, in place on the device plane `dst`; params None: the last search's."""
        f = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        check(lib().svtgpu_ccso_apply_plane(self.h, ext, plane, bit_depth, dst, dst_bits, dst_stride,
                                            None if params is None else ctypes.byref(params), ptr(f), stream))

    def close(self):
        if self.h:
            lib().svtgpu_ccso_state_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plane_sse(a, b, plane, stream=None):
    v = _U64()
    check(lib().svtgpu_plane_sse(a.h, b.h, plane, ctypes.byref(v), stream))
    return v.value


def declared_symbols(header=HEADER_PATH):
    """Function names declared in include/svtgpu.h (for the ABI export test)."""
    import re
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(svtgpu_[a-z0-9_]+)\s*\(", txt)))


def transfer_bytes(reset=False):
    """svtgpu_transfer_bytes: (host-to-device, device-to-host) bytes moved by the frame-level entry points since the
    last reset (copies and results read from mapped memory)."""
    h2d, d2h = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(lib().svtgpu_transfer_bytes(ctypes.byref(h2d), ctypes.byref(d2h), 1 if reset else 0))
    return int(h2d.value), int(d2h.value)
