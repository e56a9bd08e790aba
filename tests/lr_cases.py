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


def search_cases():
    """tests/golden/lr_search.bin: reference restoration_seg_search + rest_finish_search outputs."""
    import oracle
    g = cc.load("lr_search.bin")
    for ci in range(int(g["ncase"][0])):
        prm = [int(x) for x in g["c%d_params" % ci]]
        w, h, bd, usize, wn, sg, rdmult = prm[:7]
        ctrls = oracle.lr_controls(wn, sg, rdmult, prm[7:10], prm[10:12], prm[12:14])
        dt = np.uint16 if bd > 8 else np.uint8
        yield {
            "name": "c%d_%dx%d_bd%d_u%d_wn%d_sg%d" % (ci, w, h, bd, usize, wn, sg), "w": w, "h": h, "bd": bd,
            "unit_size": [usize, usize >> 1, usize >> 1], "ctrls": ctrls,
            "src": [g["c%d_src%d" % (ci, p)].astype(dt) for p in range(3)],
            "rec": [g["c%d_rec%d" % (ci, p)].astype(dt) for p in range(3)],
            "ftype": [int(x) for x in g["c%d_ftype" % ci]],
            "units": [rest_units_from_rows(g["c%d_units%d" % (ci, p)]) for p in range(3)],
            "sse": [g["c%d_sse%d" % (ci, p)] for p in range(3)],
            "rec_params": [g["c%d_rec%d_params" % (ci, p)] for p in range(3)],
        }


def compare_search(ft, units, recs, c):
    """Assert a search result equals the reference golden record c (frame types, unit types and the
    parameters of the chosen filters, per-unit SSEs and best parameters)."""
    assert list(ft) == c["ftype"], (c["name"], ft, c["ftype"])
    for p in range(3):
        want, got = c["units"][p], units[p]
        np.testing.assert_array_equal(got["type"], want["type"], err_msg="%s p%d types" % (c["name"], p))
        for k in range(len(want)):
            t = int(want["type"][k])
            if t == 1:
                assert list(got["vfilter"][k]) == list(want["vfilter"][k]) and \
                    list(got["hfilter"][k]) == list(want["hfilter"][k]), (c["name"], p, k)
            elif t == 2:
                assert (got["ep"][k], list(got["xqd"][k])) == (want["ep"][k], list(want["xqd"][k])), (c["name"], p, k)
        if recs is None:
            continue
        sse = np.array(recs[p]["sse"])
        sse[sse == np.iinfo(np.int64).max] = -1
        ref_sse = c["sse"][p]
        # chroma searches run only when a tool enables chroma; otherwise the reference records stay zero
        if p and not ((c["ctrls"].wn_enabled and c["ctrls"].wn_use_chroma) or
                      (c["ctrls"].sg_enabled and c["ctrls"].sg_use_chroma)):
            continue
        cols = [0] + ([1] if c["ctrls"].wn_enabled and (p == 0 or c["ctrls"].wn_use_chroma) else []) + \
            ([2] if c["ctrls"].sg_enabled and (p == 0 or c["ctrls"].sg_use_chroma) else [])
        np.testing.assert_array_equal(sse[:, cols], ref_sse[:, cols], err_msg="%s p%d sse" % (c["name"], p))
        rp = c["rec_params"][p]
        for k in range(len(rp)):
            if 2 in cols:
                assert (recs[p]["sgrproj"]["ep"][k], list(recs[p]["sgrproj"]["xqd"][k])) == \
                    (rp[k][16], [rp[k][17], rp[k][18]]), (c["name"], p, k)
            if 1 in cols and ref_sse[k][1] != -1:
                assert list(recs[p]["wiener"]["vfilter"][k][:7]) == list(rp[k][:7]) and \
                    list(recs[p]["wiener"]["hfilter"][k][:7]) == list(rp[k][8:15]), (c["name"], p, k)
