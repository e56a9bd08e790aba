"""Loop-restoration test helpers: golden decoding and synthetic unit parameters."""
import numpy as np

import cdef_cases as cc
from svtgpu import rest_units_from_rows


def frame_cases():
    g = cc.load("lr_frame.bin")
    for ci in range(int(g["ncase"][0])):
        w, h, bd, usize, mask, _ = (int(x) for x in g["c%d_params" % ci])
        dt = np.uint16 if bd > 8 else np.uint8
        yield {
            "name": "c%d_%dx%d_bd%d_u%d" % (ci, w, h, bd, usize), "w": w, "h": h, "bd": bd,
            "unit_size": [usize, usize >> 1, usize >> 1],
            "frame_type": [1 if mask >> p & 1 else 0 for p in range(3)],
            "units": [rest_units_from_rows(g["c%d_units%d" % (ci, p)]) for p in range(3)],
            "dlf": [g["c%d_dlf%d" % (ci, p)].astype(dt) for p in range(3)],
            "cdef": [g["c%d_cdef%d" % (ci, p)].astype(dt) for p in range(3)],
            "out": [g["c%d_out%d" % (ci, p)].astype(dt) for p in range(3)],
        }


def rand_wiener(r, chroma):
    lo, hi = (-5, -23, -17), (10, 8, 46)
    t = [int(r.integers(lo[k], hi[k] + 1)) for k in range(3)]
    if chroma:
        t[0] = 0
    return [t[0], t[1], t[2], -2 * sum(t), t[2], t[1], t[0], 0]


def random_units(n, seed, chroma=False, types=(0, 1, 2)):
    r = np.random.default_rng(seed)
    rows = np.zeros((n, 20), np.int32)
    for k in range(n):
        rows[k, 0] = types[int(r.integers(0, len(types)))]
        rows[k, 1:9] = rand_wiener(r, chroma)
        rows[k, 9:17] = rand_wiener(r, chroma)
        rows[k, 17] = r.integers(0, 16)
        rows[k, 18] = r.integers(-96, 32)
        rows[k, 19] = r.integers(-32, 96)
    return rest_units_from_rows(rows)
