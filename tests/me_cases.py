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
