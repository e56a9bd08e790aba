"""CCSO test helpers: the reference's goldens (tests/golden/ccso.bin, oracle/ref_harness/
gen_golden_ccso.c over the fork's own EbCcso.c / EbPickccso.c) unpacked into the layouts the entry points take."""
import numpy as np

import cdef_cases as cc


def golden():
    return cc.load("ccso.bin")


def full(plane, w, h):
    """A (ph, pw) plane into an (h, w) uint16 array (stride w, the plane in the top-left): the ccso_stride layout."""
    a = np.zeros((h, w), np.uint16)
    a[:plane.shape[0], :plane.shape[1]] = plane
    return a


def params(g, tag, n, p):
    from svtgpu import CcsoParams
    return CcsoParams.make(g["%s_prm%d_%d" % (tag, n, p)][:6], g["%s_lut%d_%d" % (tag, n, p)])


def search_cases(g):
    """dicts: w, h, bd, q, rdmult, bias, org / rec (3 full arrays), pre, ext (when recorded), params / flags (expected,
    3 each), frame_flag, out (3 planes, 8-bit cases)"""
    out = []
    for n, m in enumerate(g["srch_meta"]):
        w, h, bd, q, rdmult, bias = (int(v) for v in m)
        c = dict(n=n, w=w, h=h, bd=bd, q=q, rdmult=rdmult, bias=bias)
        c["org"] = [full(g["srch_org%d_%d" % (n, p)], w, h) for p in range(3)]
        c["rec"] = [full(g["srch_rec%d_%d" % (n, p)], w, h) for p in range(3)]
        c["pre"] = g["srch_pre%d" % n].astype(np.uint16)
        c["ext"] = g.get("srch_ext%d" % n)
        c["params"] = [params(g, "srch", n, p) for p in range(3)]
        c["flags"] = [g["srch_flags%d_%d" % (n, p)] for p in range(3)]
        c["frame_flag"] = int(g["srch_frame_flag%d" % n][0])
        c["out"] = [g["srch_out%d_%d" % (n, p)] for p in range(3)] if bd == 8 else None
        out.append(c)
    return out


def apply_cases(g):
    """dicts: w, h, pre (uint8), inp / out (3 uint8 planes), params / flags (3 each)"""
    out = []
    for n, m in enumerate(g["app_meta"]):
        w, h = (int(v) for v in m)
        out.append(dict(n=n, w=w, h=h, pre=g["app_pre%d" % n], inp=[g["app_in%d_%d" % (n, p)] for p in range(3)],
                        out=[g["app_out%d_%d" % (n, p)] for p in range(3)],
                        params=[params(g, "app", n, p) for p in range(3)],
                        flags=[g["app_flags%d_%d" % (n, p)] for p in range(3)]))
    return out


BLK_FIELDS = ("pw", "ph", "x", "y", "hs", "vs", "blk", "bd", "sup", "qs", "clf", "bo", "band_log2", "es", "cs", "loc0")


def block_cases(g):
    out = []
    for n, m in enumerate(g["blk_meta"]):
        c = dict(zip(BLK_FIELDS, (int(v) for v in m)))
        c.update(n=n, ext=g["blk_ext%d" % n], cls0=g["blk_cls0_%d" % n], cls1=g["blk_cls1_%d" % n],
                 lut=g["blk_lut%d" % n], dst0=g["blk_dst0_%d" % n], with_buf=g["blk_with%d" % n],
                 wo_buf=g["blk_wo%d" % n], ssd=int(g["blk_ssd%d" % n][0]))
        out.append(c)
    return out


def sample_pos(stride, sup):
    """derive_ccso_sample_pos (EbCcso.c:204-234)"""
    return [(-stride, stride), (-stride - 1, stride + 1), (-1, 1), (stride - 1, -stride + 1), (-3, 3), (-5, 5)][sup]


def content(w, h, bd, seed):
    """smooth org, rec = org + a band / edge biased error (the golden generator's model, numpy)"""
    rng = np.random.default_rng(seed)
    maxv, sh = (1 << bd) - 1, bd - 8
    org, rec = [], []
    for p in range(3):
        pw, ph = (w >> 1, h >> 1) if p else (w, h)
        kn = rng.integers(0, 256, size=(ph // 16 + 2, pw // 16 + 2)).astype(np.float64)
        ys, xs = np.arange(ph) / 16.0, np.arange(pw) / 16.0
        gy, gx = np.floor(ys).astype(int), np.floor(xs).astype(int)
        fy, fx = (ys - gy)[:, None], (xs - gx)[None, :]
        v = (kn[gy][:, gx] * (1 - fx) * (1 - fy) + kn[gy][:, gx + 1] * fx * (1 - fy) +
             kn[gy + 1][:, gx] * (1 - fx) * fy + kn[gy + 1][:, gx + 1] * fx * fy)
        v[:, : pw // 8] /= 16
        v[:, pw - pw // 8:] = 255 - (255 - v[:, pw - pw // 8:]) / 16
        o = np.clip((v.astype(np.int64) << sh) + rng.integers(-2 << sh, 3 << sh, size=v.shape), 0, maxv)
        gxd = np.zeros_like(o)
        gxd[:, :-1] = o[:, 1:] - o[:, :-1]
        e = rng.integers(-3, 4, size=o.shape) - 2 * (o > maxv * 3 // 4) + 2 * (gxd > (8 << sh)) - 2 * (gxd < -(8 << sh))
        r = np.clip(o + (e << sh), 0, maxv)
        org.append(full(o.astype(np.uint16), w, h))
        rec.append(full(r.astype(np.uint16), w, h))
    pre = np.clip(rec[0].astype(np.int64) + rng.integers(-1, 2, size=(h, w)), 0, maxv).astype(np.uint16)
    return org, rec, pre
