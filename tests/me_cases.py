"""Open-loop ME test helpers: the reference goldens (tests/golden/me_sad.bin, oracle/ref_harness/gen_golden_me.c)."""
import numpy as np

import cdef_cases as cc


def golden():
    return cc.load("me_sad.bin")


def frames(g):
    """Per golden frame case: (src, [ref0, ref1], origin [nsb][2][2], saw, sah, sub, best_sad, best_mv)."""
    out = []
    for n, (W, H, saw, sah, sub, nref) in enumerate(g["frame_meta"]):
        nsb = (W // 64) * (H // 64)
        out.append((g["src%d" % n], [g["ref%d_%d" % (n, q)] for q in range(nref)],
                    g["origin%d" % n].reshape(nsb, nref, 2), int(saw), int(sah), int(sub),
                    g["best_sad%d" % n].reshape(nsb, nref, 85), g["best_mv%d" % n].reshape(nsb, nref, 85)))
    return out


def loop_cases(g):
    """sad_loop golden calls: (src, ref, meta) with meta = bw, bh, saw, sah, ss, rs, srr, skip, best, xc | yc << 16."""
    return [(g["loop_src%d" % n], g["loop_ref%d" % n], [int(v) for v in g["loop_meta"][n]])
            for n in range(len(g["loop_meta"]))]


import ctypes


class MvCostParams(ctypes.Structure):
    """The reference's MV_COST_PARAMS (mcomp.h:37-48), x86-64 layout."""
    _fields_ = [("ref_mv", ctypes.c_void_p), ("full_ref_mv", ctypes.c_int16 * 2), ("mv_cost_type", ctypes.c_uint8),
                ("mvjcost", ctypes.c_void_p), ("mvcost", ctypes.c_void_p * 2), ("error_per_bit", ctypes.c_int),
                ("early_exit_th", ctypes.c_int), ("sad_per_bit", ctypes.c_int)]


def pme_cases(g):
    """Per golden call: (params struct, keep-alive arrays, src, ref, meta list) -- meta as gen_golden_me.c writes it:
    bw, bh, saw, sah, step, ss, rs, rows, ref_row, ref_col, best_in, type, epb, sx, sy, mvx, mvy, best, bx, by."""
    jc = np.ascontiguousarray(g["pme_jc"], np.int32)
    tab = np.ascontiguousarray(g["pme_tab"], np.int32)
    out = []
    for n, m in enumerate(g["pme_meta"]):
        m = [int(v) for v in m]
        ref_mv = np.array([m[8], m[9]], np.int16)
        p = MvCostParams()
        p.ref_mv = ref_mv.ctypes.data
        p.mv_cost_type = m[11]
        p.mvjcost = jc.ctypes.data
        p.mvcost[0] = tab[0].ctypes.data + 4 * (1 << 14)
        p.mvcost[1] = tab[1].ctypes.data + 4 * (1 << 14)
        p.error_per_bit = m[12]
        out.append((p, (ref_mv, jc, tab), g["pme_src%d" % n], g["pme_ref%d" % n], m))
    return out
