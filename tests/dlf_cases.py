"""Deblocking test cases: golden-fixture decoding and synthetic mode-info / frame generators."""
import numpy as np

import cdef_cases as cc
from svtgpu import LfParams, LF_MI_DTYPE

LPF_NAMES = ["horizontal_4", "horizontal_6", "horizontal_8", "horizontal_14",
             "vertical_4", "vertical_6", "vertical_8", "vertical_14"]


def frame_cases():
    """Yield dicts from tests/golden/dlf_frame.bin (reference svt_av1_loop_filter_frame outputs)."""
    g = cc.load("dlf_frame.bin")
    for ci in range(int(g["ncase"][0])):
        prm = g["c%d_params" % ci].astype(int)
        w, h, bd, pipe16, ps, pe, fl0, fl1, flu, flv, sharp, mrd, seg = prm[:13]
        en = prm[23:87].reshape(8, 8)
        data = prm[87:151].reshape(8, 8)
        p = LfParams.make(fl0, fl1, flu, flv, sharp,
                          ref_deltas=prm[13:21] if mrd else None, mode_deltas=prm[21:23] if mrd else None,
                          seg_enabled=en if seg else None, seg_data=data if seg else None)
        dt = np.uint16 if bd > 8 else np.uint8
        pad = [int(x) for x in g["c%d_pad" % ci]] if ("c%d_pad" % ci) in g else [0, 0]
        yield {
            "name": "c%d_%dx%d_bd%d%s%s" % (ci, w, h, bd, "_p16" if pipe16 else "",
                                           "_crop%dx%d" % (w - pad[0], h - pad[1]) if any(pad) else ""),
            "w": int(w), "h": int(h), "bd": int(bd), "plane_start": int(ps), "plane_end": int(pe),
            "crop": (int(w - pad[0]), int(h - pad[1])),
            "params": p,
            "mi": np.ascontiguousarray(g["c%d_mi" % ci]).view(LF_MI_DTYPE).reshape(g["c%d_mi" % ci].shape[:2]),
            "inp": [g["c%d_in%d" % (ci, k)].astype(dt) for k in range(3)],
            "out": [g["c%d_out%d" % (ci, k)].astype(dt) for k in range(3)],
        }


# block sizes (BlockSize enum order, EbDefinitions.h) and the partition generator used by the tests
BW = [4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 32, 64, 64, 64, 128, 128, 4, 16, 8, 32, 16, 64]
BH = [4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 64, 32, 64, 128, 64, 128, 16, 4, 32, 8, 64, 16]
_BS = {(w, h): b for b, (w, h) in enumerate(zip(BW, BH))}


def random_mode_info(width, height, seed, p_skip=0.5, p_intra=0.3, segments=False, sb=64, min_block=4,
                     rect128=False):
    """Random partition of each SB into AV1 block shapes with random tx depth / skip / refs / modes.
    rect128 (sb=128): 128x64 and 64x128 blocks besides 128x128."""
    rng = np.random.default_rng(seed)
    mr, mc = ((height + 7) & ~7) >> 2, ((width + 7) & ~7) >> 2
    mi = np.zeros((mr, mc), LF_MI_DTYPE)

    def place(r, c, bw, bh):
        if r >= mr or c >= mc:
            return
        inter = rng.random() >= p_intra
        rec = (_BS[(bw, bh)], rng.integers(0, 3), int(rng.random() < p_skip),
               int(rng.integers(1, 8)) if inter else 0,
               int(rng.integers(13, 25)) if inter else int(rng.integers(0, 13)),
               int(rng.integers(0, 8)) if segments else 0, (0, 0))
        mi[r:r + bh // 4, c:c + bw // 4] = rec

    def part(r, c, s):
        if r >= mr or c >= mc:
            return
        q = s // 4
        opt = int(rng.integers(0, 8 if s >= 64 else 6))
        if s >= 64 and opt >= 6:
            opt = 3
        if s == 8 and (opt >= 4 or min_block > 4):
            opt = 0 if min_block > 4 else int(rng.integers(0, 4))
        if opt == 0:
            place(r, c, s, s)
        elif opt == 1:
            place(r, c, s, s // 2), place(r + q // 2, c, s, s // 2)
        elif opt == 2:
            place(r, c, s // 2, s), place(r, c + q // 2, s // 2, s)
        elif opt == 3:
            if s == 8:
                for k in range(4):
                    place(r + (k >> 1), c + (k & 1), 4, 4)
            else:
                for k in range(4):
                    part(r + (k >> 1) * q // 2, c + (k & 1) * q // 2, s // 2)
        elif opt == 4:
            for k in range(4):
                place(r + k * q // 4, c, s, s // 4)
        else:
            for k in range(4):
                place(r, c + k * q // 4, s // 4, s)

    for r in range(0, mr, sb // 4):
        for c in range(0, mc, sb // 4):
            u = rng.random() if sb == 128 else 1.0
            if rect128 and 0.2 <= u < 0.3:
                place(r, c, 128, 64), place(r + 16, c, 128, 64)
            elif rect128 and 0.3 <= u < 0.4:
                place(r, c, 64, 128), place(r, c + 16, 64, 128)
            elif u < (0.2 if rect128 else 0.3):
                place(r, c, 128, 128)
            else:
                for k in range(4 if sb == 128 else 1):
                    part(r + (k >> 1) * 16, c + (k & 1) * 16, 64)
    return mi
