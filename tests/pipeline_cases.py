"""Whole-frame pipeline cases (DLF pick + filter -> CDEF search + pick + apply -> LR search + apply).

Each case fixes a picture size / bit depth, the encoder's per-level controls (cdef_level, dlf_level, wn/sg
filter levels: the reference's EncModeConfig.c tables), the frame header inputs the path reads (base_q_idx,
starting loop-filter levels, sharpness, mode/ref deltas, temporal layer, frame/update type for the CDEF
lambda) and a mode-info grid.  tests/golden/make_pipeline_golden.py runs the reference's own frame-level
code on them (oracle/_ref/gen_golden_pipe) and stores the outputs — full arrays for the small cases, SHA-256
digests of the planes and search tables for the 1080p 8-bit and 4K 10-bit configurations of BASELINE.json.

The inputs are generated here with integer-only numpy operations (PCG64 integer draws, integer arithmetic) so
they are bit-identical on every host; each fixture also stores the SHA-256 of its inputs and the tests check it
before comparing anything.
"""
import hashlib
import os

import numpy as np

import dlf_cases

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAGIC = 0x45504950
HEADER = ["magic", "w", "h", "bd", "q", "cdef_level", "dlf_level", "wn_level", "sg_level", "lf0", "lf1", "lfu", "lfv",
          "sharp", "mrd", "tl", "frame_type", "update_type", "hier", "rdmult", "sw0", "sw1", "sw2", "wc0", "wc1", "sc0",
          "sc1", "us_y", "us_uv", "cdef_sc", "cdef_sr", "rest_sc", "rest_sr", "only4x4", "sb", "pred_y", "pred_uv",
          "mesad", "in_res", "slice"]
HEADER_WORDS = 64
KEY_FRAME, INTER_FRAME = 0, 1
KF_UPDATE, LF_UPDATE, GF_UPDATE, ARF_UPDATE, INTNL_ARF_UPDATE = 0, 1, 2, 3, 6

# the bench's rate inputs (bench.py) and defaults shared by the cases
_BASE = dict(q=160, cdef_level=1, dlf_level=1, wn_level=1, sg_level=1, lf=(16, 16, 8, 8), sharp=0, mrd=0,
             ref_deltas=(1, 0, 0, 0, -1, 0, -1, -1), mode_deltas=(0, 0), tl=0, frame_type=INTER_FRAME,
             update_type=ARF_UPDATE, hier=3, rdmult=7000, sw=(300, 700, 900), wc=(250, 800), sc=(250, 900),
             us=(64, 32), cdef_seg=(1, 1), rest_seg=(1, 1), only4x4=0, sb=64, pred=(0, 0),
             mi=("random", 1, 0.3), seed=1, digest=False, mesad=0, in_res=0, slice=0)
B_SLICE, P_SLICE, I_SLICE = 0, 1, 2


def _case(**kw):
    c = dict(_BASE)
    c.update(kw)
    return c


CASES = {
    # small frames: every output array is stored
    "mini8": _case(w=256, h=144, bd=8, q=120, lf=(8, 8, 4, 4), mi=("random", 11, 0.3), seed=101, tl=3,
                   update_type=LF_UPDATE),
    "mini10": _case(w=320, h=200, bd=10, q=180, cdef_level=2, dlf_level=2, wn_level=2, sg_level=2, lf=(20, 20, 10, 12),
                    sharp=2, mrd=1, ref_deltas=(1, 0, 0, 0, -1, 0, -1, -1), mode_deltas=(-2, 3), tl=1,
                    update_type=INTNL_ARF_UPDATE, us=(128, 64), cdef_seg=(2, 2), rest_seg=(2, 2),
                    mi=("random", 12, 0.2), seed=102),
    "mini10b": _case(w=200, h=136, bd=10, q=90, cdef_level=9, wn_level=3, sg_level=3, lf=(12, 30, 6, 0), only4x4=1,
                     mi=("random", 13, 0.5), seed=103),
    "mini8c": _case(w=136, h=264, bd=8, q=220, cdef_level=12, dlf_level=2, wn_level=4, sg_level=4, lf=(40, 40, 20, 20),
                    tl=2, frame_type=KEY_FRAME, update_type=KF_UPDATE, mi=("random", 14, 0.1), seed=104),
    "mini8d": _case(w=264, h=136, bd=8, q=40, cdef_level=16, wn_level=5, sg_level=0, lf=(4, 4, 2, 2),
                    us=(128, 128), mi=("random", 15, 0.6), seed=105),
    "mini10e": _case(w=192, h=128, bd=10, q=255, cdef_level=5, wn_level=0, sg_level=2, lf=(63, 50, 40, 30), sharp=7,
                     tl=4, update_type=LF_UPDATE, mi=("random", 16, 0.0), seed=106),
    # SB128 mode-info (128x128 / 128x64 / 64x128 blocks): the search skips the odd 64x64 halves (EbCdefProcess.c:193)
    "sb128_10": _case(w=384, h=256, bd=10, q=140, sb=128, mi=("random128", 17, 0.3), seed=107),
    "sb128_8": _case(w=320, h=200, bd=8, q=100, sb=128, cdef_level=3, mi=("random128", 18, 0.2), seed=108),
    # reference filter strengths (use_reference_cdef_fs): no search, strengths from the MDC prediction
    "reffs_10": _case(w=256, h=192, bd=10, q=150, cdef_level=17, pred=(9, 6), mi=("random", 19, 0.4), seed=109),
    "reffs_8": _case(w=200, h=136, bd=8, q=60, cdef_level=11, pred=(0, 0), mi=("random", 20, 0.4), seed=110),
    # the SB-based DLF levels 3/4/5 (presets M6 and up, EncModeConfig.c:1516-1609): LPF_PICK_FROM_Q levels and the
    # encode loop's per-SB filter (EbCodingLoop.c:2260-2281) -- ME distortions above / between / below the
    # zero-strength thresholds (disable_dlf_th, EbDeblockingFilter.c:26) of the level and resolution class
    "sbdlf10": _case(w=320, h=200, bd=10, q=150, dlf_level=3, mesad=5000, in_res=1, mi=("random", 21, 0.3), seed=111),
    "sbdlf8_128": _case(w=384, h=256, bd=8, q=200, dlf_level=4, sb=128, mesad=20000, in_res=0, tl=1,
                        mi=("random128", 22, 0.2), seed=112),
    "sbdlf10_zero": _case(w=136, h=96, bd=10, q=60, dlf_level=4, mesad=100, in_res=0, mi=("random", 25, 0.3),
                          seed=115),
    "sbdlf10_uv0": _case(w=256, h=192, bd=10, q=120, dlf_level=5, mesad=7000, in_res=0, mi=("random", 23, 0.4),
                         seed=113),
    "sbdlf8_key": _case(w=200, h=136, bd=8, q=90, dlf_level=3, frame_type=KEY_FRAME, update_type=KF_UPDATE,
                        slice=I_SLICE, mesad=0, mi=("random", 24, 0.3), seed=114),
    # BASELINE.json configs[1] (1080p 8-bit) and configs[2] (4K 10-bit, the bench workload): digests only
    "c1_1080p8": _case(w=1920, h=1080, bd=8, us=(256, 128), mi=("bench", 0x5EED0002), seed=0x5EED0002,
                       digest=True),
    "c3_4k10": _case(w=3840, h=2160, bd=10, us=(256, 128), mi=("bench", 0x5EED0003), seed=0x5EED0003, digest=True),
}
SMALL = [k for k, c in CASES.items() if not c["digest"]]


def frame_pair(w, h, bd, seed):
    """The integer-only generator (synth.frame_pair_int, shared with bench.py)."""
    import synth
    return synth.frame_pair_int(w, h, bd, seed)


def mode_info(c):
    kind = c["mi"][0]
    if kind == "bench":
        import synth
        return synth.mode_info(c["w"], c["h"], 3)
    seed, p_skip = c["mi"][1], c["mi"][2]
    if kind == "random128":
        return dlf_cases.random_mode_info(c["w"], c["h"], seed, p_skip=p_skip, sb=128, rect128=True)
    return dlf_cases.random_mode_info(c["w"], c["h"], seed, p_skip=p_skip)


def inputs(name):
    """(source planes, recon planes, mode info) of a case."""
    c = CASES[name]
    src, rec = frame_pair(c["w"], c["h"], c["bd"], c["seed"])
    return src, rec, mode_info(c)


def input_digest(src, rec, mi):
    h = hashlib.sha256()
    for a in list(src) + list(rec):
        h.update(np.ascontiguousarray(a, np.uint16).tobytes())
    h.update(np.ascontiguousarray(mi).view(np.uint8).tobytes())
    return h.hexdigest()


def header(c):
    v = dict(magic=MAGIC, w=c["w"], h=c["h"], bd=c["bd"], q=c["q"], cdef_level=c["cdef_level"],
             dlf_level=c["dlf_level"], wn_level=c["wn_level"], sg_level=c["sg_level"], lf0=c["lf"][0], lf1=c["lf"][1],
             lfu=c["lf"][2], lfv=c["lf"][3], sharp=c["sharp"], mrd=c["mrd"], tl=c["tl"], frame_type=c["frame_type"],
             update_type=c["update_type"], hier=c["hier"], rdmult=c["rdmult"], sw0=c["sw"][0], sw1=c["sw"][1],
             sw2=c["sw"][2], wc0=c["wc"][0], wc1=c["wc"][1], sc0=c["sc"][0], sc1=c["sc"][1], us_y=c["us"][0],
             us_uv=c["us"][1], cdef_sc=c["cdef_seg"][0], cdef_sr=c["cdef_seg"][1], rest_sc=c["rest_seg"][0],
             rest_sr=c["rest_seg"][1], only4x4=c["only4x4"], sb=c["sb"], pred_y=c["pred"][0], pred_uv=c["pred"][1],
             mesad=c["mesad"], in_res=c["in_res"], slice=c["slice"])
    hdr = np.zeros(HEADER_WORDS, np.int32)
    for i, k in enumerate(HEADER):
        hdr[i] = v[k]
    return hdr


def write_input(path, name, src, rec, mi):
    """Input file of gen_golden_pipe: header int32[64], int8 ref_deltas[8] mode_deltas[2] pad[6], source Y U V and
    recon Y U V as uint16, the mode-info grid as SvtGpuLfMi records."""
    c = CASES[name]
    d = np.zeros(16, np.int8)
    d[:8] = c["ref_deltas"]
    d[8:10] = c["mode_deltas"]
    with open(path, "wb") as f:
        f.write(header(c).tobytes())
        f.write(d.tobytes())
        for a in list(src) + list(rec):
            f.write(np.ascontiguousarray(a, np.uint16).tobytes())
        f.write(np.ascontiguousarray(mi).view(np.uint8).tobytes())


def is_frame_key(k):
    return k[:3] in ("dlf", "cde", "lr0", "lr1", "lr2") and k[-1].isdigit() and not k.startswith(("lr_", "cdef_"))


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(name):
    """The stored reference outputs of a case (np.load, no pickle)."""
    with np.load(os.path.join(GOLDEN, "pipe_%s.npz" % name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def cdef_mask(mi):
    """Per-8x8 'listed' mask of svt_sb_compute_cdef_list (EbEncCdef.c:238): any of the four 4x4 mi non-skip."""
    s = np.ascontiguousarray(mi)["skip"].astype(bool)
    mr, mc = s.shape
    s = s[:mr & ~1, :mc & ~1]
    return (~(s[0::2, 0::2] & s[0::2, 1::2] & s[1::2, 0::2] & s[1::2, 1::2])).astype(np.uint8)


def lf_params(c):
    from svtgpu import LfParams
    lf = c["lf"]
    if c["mrd"]:
        return LfParams.make(lf[0], lf[1], lf[2], lf[3], c["sharp"], ref_deltas=c["ref_deltas"],
                             mode_deltas=c["mode_deltas"])
    return LfParams.make(lf[0], lf[1], lf[2], lf[3], c["sharp"])
