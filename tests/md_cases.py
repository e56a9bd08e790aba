"""MD distortion test helpers: golden decoding and synthetic motion-vector fields."""
import numpy as np

import cdef_cases as cc

MD_SIZES = [(4, 4), (4, 8), (8, 4), (8, 8), (8, 16), (16, 8), (16, 16), (16, 32), (32, 16), (32, 32), (32, 64),
            (64, 32), (64, 64), (64, 128), (128, 64), (128, 128), (4, 16), (16, 4), (8, 32), (32, 8), (16, 64),
            (64, 16)]


def golden():
    return cc.load("md_dist.bin")


def case(g, si, c):
    """(src16, ref16, src8, ref8) of golden case c of size si (8-bit kernels saw the low byte; case 1 is the
    maximum-difference pattern 255/0)."""
    # copies: golden records are packed at arbitrary byte offsets, and the highbd kernels' pointer encoding
    # (CONVERT_TO_BYTEPTR, address >> 1) needs 2-byte aligned planes
    s16, r16 = g["s%d_src" % si][c].copy(), g["s%d_ref" % si][c].copy()
    if c == 1:
        return s16, r16, np.full(s16.shape, 255, np.uint8), np.zeros(r16.shape, np.uint8)
    return s16, r16, (s16 & 255).astype(np.uint8), (r16 & 255).astype(np.uint8)


def mvs(width, height, nref, seed, rng_max=16):
    nsb = ((width + 63) // 64) * ((height + 63) // 64)
    r = np.random.default_rng(seed)
    return r.integers(-rng_max, rng_max + 1, size=(nsb, nref, 2)).astype(np.int16)


def ref_frames(width, height, bd, nref, seed):
    """Independent synthetic luma planes (same generator as the source, different seeds)."""
    import synth
    out = []
    for r in range(nref):
        s, _ = synth.frame_pair(width, height, bd, seed=seed + 17 * (r + 1))
        out.append(s[0])
    return out
